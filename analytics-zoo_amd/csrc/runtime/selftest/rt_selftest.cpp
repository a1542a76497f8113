// Standalone self-test of the host runtime (csrc/runtime/*.cpp) for sanitizer builds.
//
// tools/sanitize_runtime.py compiles this file with -DZOO_RT_NO_PYTHON (no pybind11, no
// interpreter, so no preloaded sanitizer runtime is needed) under
//   asan  : -fsanitize=address,undefined -fno-sanitize-recover=all
//   tsan  : -fsanitize=thread
// and runs it. Every section drives the same code the Python extension runs: the serving
// queue (Store command set, blocking read_batch/finish fast path, the RESP TCP front end),
// the minibatch Gatherer, CRC32C/TFRecord framing and the protobuf wire scanner, with
// concurrent producers/consumers and randomly mutated inputs. Reference parity for the
// same pieces is covered by the Python tests (tests/test_serving*.py, test_runtime*.py);
// this binary only has to finish without a sanitizer report and with every check true.
#define ZOO_RT_NO_PYTHON 1
#include "../runtime.cpp"
#include "../serving.cpp"

#include <cstdio>
#include <cstdlib>
#include <random>

using zoo_serving::Reply;
using zoo_serving::Server;
using zoo_serving::Store;

static int g_fail = 0;
#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                   \
    }                                                             \
  } while (0)

static std::vector<std::string> V(std::initializer_list<std::string> l) { return std::vector<std::string>(l); }

static std::string b64(const std::string& in) {
  static const char* T = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string o;
  size_t i = 0;
  for (; i + 2 < in.size(); i += 3) {
    const unsigned v = ((unsigned char)in[i] << 16) | ((unsigned char)in[i + 1] << 8) | (unsigned char)in[i + 2];
    o += T[v >> 18]; o += T[(v >> 12) & 63]; o += T[(v >> 6) & 63]; o += T[v & 63];
  }
  if (i + 1 == in.size()) {
    const unsigned v = (unsigned char)in[i] << 16;
    o += T[v >> 18]; o += T[(v >> 12) & 63]; o += "==";
  } else if (i + 2 == in.size()) {
    const unsigned v = ((unsigned char)in[i] << 16) | ((unsigned char)in[i + 1] << 8);
    o += T[v >> 18]; o += T[(v >> 12) & 63]; o += T[(v >> 6) & 63]; o += '=';
  }
  return o;
}

// ------------------------------------------------------------------ crc / tfrecord
static uint32_t crc_bitwise(const uint8_t* p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) {
    c ^= p[i];
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
  }
  return c ^ 0xFFFFFFFFu;
}

static void test_crc() {
  const char* s = "123456789";
  CHECK(crc32c_raw(reinterpret_cast<const uint8_t*>(s), 9) == 0xE3069283u);  // RFC 3720 check value
  std::mt19937 rng(1);
  std::vector<std::thread> ts;
  std::atomic<int> bad{0};
  for (int t = 0; t < 4; ++t)  // concurrent first use of the table
    ts.emplace_back([&, t] {
      std::mt19937 r(t);
      for (int it = 0; it < 200; ++it) {
        std::string b(r() % 300, '\0');
        for (auto& c : b) c = (char)r();
        const size_t off = b.empty() ? 0 : r() % b.size();  // unaligned starts
        const uint8_t* p = reinterpret_cast<const uint8_t*>(b.data()) + off;
        if (crc32c_raw(p, b.size() - off) != crc_bitwise(p, b.size() - off)) ++bad;
      }
    });
  for (auto& t : ts) t.join();
  CHECK(bad == 0);
  const std::string payload = "tensorboard event";
  const std::string f = tfrecord_frame_raw(payload);
  CHECK(f.size() == 12 + payload.size() + 4);
  uint64_t len;
  std::memcpy(&len, f.data(), 8);
  CHECK(len == payload.size());
  uint32_t dc;
  std::memcpy(&dc, f.data() + 12 + payload.size(), 4);
  CHECK(dc == mask_crc(crc32c_raw(reinterpret_cast<const uint8_t*>(payload.data()), payload.size())));
  CHECK(tfrecord_frame_raw("").size() == 16);
}

// ------------------------------------------------------------------ protobuf scanner
static void put_varint(std::string* o, uint64_t v) {
  while (v >= 0x80) { o->push_back((char)(v | 0x80)); v >>= 7; }
  o->push_back((char)v);
}

static void test_pb() {
  std::string m;
  put_varint(&m, (1 << 3) | 0); put_varint(&m, 300);
  put_varint(&m, (2 << 3) | 2); put_varint(&m, 5); m += "hello";
  put_varint(&m, (3 << 3) | 5); m.append("\x01\x00\x00\x00", 4);
  put_varint(&m, (4 << 3) | 1); m.append("\x02\x00\x00\x00\x00\x00\x00\x00", 8);
  put_varint(&m, (5 << 3) | 0); put_varint(&m, ~0ull);
  std::vector<PbField> fs;
  pb_scan(reinterpret_cast<const uint8_t*>(m.data()), m.size(), &fs);
  CHECK(fs.size() == 5);
  if (fs.size() == 5) {
    CHECK(fs[0].field == 1 && fs[0].v == 300);
    CHECK(fs[1].wt == 2 && m.substr(fs[1].off, fs[1].v) == "hello");
    CHECK(fs[2].v == 1 && fs[3].v == 2 && fs[4].v == ~0ull);
  }
  // mutated / truncated / random inputs: scan or throw, never read out of bounds
  std::mt19937 rng(7);
  int ok = 0, thrown = 0;
  for (int it = 0; it < 20000; ++it) {
    std::string b = m;
    if (it & 1) {
      b.resize(rng() % 64);
      for (auto& c : b) c = (char)rng();
    } else {
      for (int k = 0; k < 3; ++k) b[rng() % b.size()] = (char)rng();
      b.resize(rng() % (b.size() + 1));
    }
    // heap copy of exactly b.size() bytes so ASan sees any overread
    std::unique_ptr<uint8_t[]> buf(new uint8_t[b.size() + 1]);
    std::memcpy(buf.get(), b.data(), b.size());
    std::vector<PbField> out;
    try {
      pb_scan(buf.get(), b.size(), &out);
      for (auto& f : out)
        if (f.wt == 2) CHECK(f.off + f.v <= b.size());
      ++ok;
    } catch (const std::runtime_error&) {
      ++thrown;
    }
  }
  CHECK(ok > 0 && thrown > 0);
}

// ------------------------------------------------------------------ gatherer
static void test_gatherer() {
  const int64_t nrows = 1000, rb = 24;
  std::vector<char> src(nrows * rb);
  for (int64_t r = 0; r < nrows; ++r)
    for (int64_t j = 0; j < rb; ++j) src[r * rb + j] = (char)(r * 7 + j);
  Gatherer g(4);
  std::vector<std::thread> prod;
  std::atomic<int> bad{0};
  for (int t = 0; t < 3; ++t)
    prod.emplace_back([&, t] {
      std::mt19937 rng(t + 11);
      for (int it = 0; it < 50; ++it) {
        const int64_t n = 1 + rng() % 700;
        std::vector<int64_t> idx(n);
        for (auto& i : idx) i = rng() % nrows;
        std::vector<char> dst(n * rb);
        const int64_t tk = g.submit((uintptr_t)src.data(), nrows, rb, (uintptr_t)idx.data(), n, (uintptr_t)dst.data());
        g.wait(tk);
        if (!g.ready(tk)) ++bad;
        for (int64_t i = 0; i < n; ++i)
          if (std::memcmp(&dst[i * rb], &src[idx[i] * rb], rb) != 0) ++bad;
      }
    });
  for (auto& t : prod) t.join();
  CHECK(bad == 0);
  std::vector<int64_t> badidx{0, nrows};
  std::vector<char> dst(2 * rb);
  bool threw = false;
  try {
    g.gather((uintptr_t)src.data(), nrows, rb, (uintptr_t)badidx.data(), 2, (uintptr_t)dst.data());
  } catch (const std::out_of_range&) {
    threw = true;
  }
  CHECK(threw);
}

// ------------------------------------------------------------------ store commands
static void test_store_commands() {
  Store st((size_t)1 << 30);
  CHECK(st.exec(V({"PING"})).s == "PONG");
  CHECK(st.exec(V({"xadd", "s", "*", "uri", "a", "image", b64("abc")})).k == Reply::BULK);
  CHECK(st.exec(V({"XADD", "s", "MAXLEN", "~", "5", "*", "uri", "b"})).k == Reply::BULK);
  CHECK(st.exec(V({"XLEN", "s"})).i == 2);
  CHECK(st.exec(V({"XGROUP", "CREATE", "s", "g", "0"})).s == "OK");
  CHECK(st.exec(V({"XGROUP", "CREATE", "s", "g", "0"})).k == Reply::ERR);
  Reply r = st.exec(V({"XREADGROUP", "GROUP", "g", "c", "COUNT", "10", "STREAMS", "s", ">"}));
  CHECK(r.k == Reply::ARR && r.a.size() == 1 && r.a[0].a[1].a.size() == 2);
  CHECK(st.exec(V({"HSET", "h", "f", "v", "f2", "v2"})).i == 2);
  CHECK(st.exec(V({"HGET", "h", "f"})).s == "v");
  CHECK(st.exec(V({"HGETALL", "h"})).a.size() == 4);
  CHECK(st.exec(V({"KEYS", "*"})).a.size() == 2);
  CHECK(st.exec(V({"XADD", "h", "*", "x", "y"})).k == Reply::ERR);  // WRONGTYPE
  CHECK(st.exec(V({"CONFIG", "SET", "maxmemory", "1k"})).k != Reply::ERR);
  for (int i = 0; i < 100; ++i) st.exec(V({"XADD", "s", "*", "uri", std::to_string(i), "image", std::string(100, 'A')}));
  CHECK(st.exec(V({"XLEN", "s"})).i < 100);  // memory-based trim kept it under 1 KiB
  CHECK(st.exec(V({"DEL", "h", "nope"})).i == 1);
  CHECK(st.exec(V({"FLUSHALL"})).s == "OK");
  CHECK(st.exec(V({"DBSIZE"})).i == 0);
  CHECK(st.exec(V({})).k == Reply::ERR);

  // random command fuzz: wrong arity, bad ids, bad numbers -> error replies, no crash
  const char* cmds[] = {"XADD", "XLEN", "XTRIM", "XRANGE", "XGROUP", "XACK", "XDEL", "HSET", "HMSET", "HGET",
                        "HGETALL", "KEYS", "DEL", "EXISTS", "INFO", "CONFIG", "DBSIZE", "ECHO", "PING",
                        "XREADGROUP", "FLUSHDB"};
  const char* words[] = {"s", "h", "g", "c", "*", ">", "$", "0", "0-1", "-", "+", "1-x", "MAXLEN", "~", "99999999999999999999",
                         "-5", "COUNT", "BLOCK", "STREAMS", "GROUP", "CREATE", "DESTROY", "SET", "GET", "maxmemory",
                         "uri", "image", "!!", ""};
  std::mt19937 rng(3);
  int errs = 0;
  for (int it = 0; it < 20000; ++it) {
    std::vector<std::string> a{cmds[rng() % (sizeof(cmds) / sizeof(*cmds))]};
    if (a[0] == "XREADGROUP") continue;  // covered below with a bounded BLOCK
    const int n = rng() % 8;
    for (int k = 0; k < n; ++k) a.push_back(words[rng() % (sizeof(words) / sizeof(*words))]);
    if (st.exec(a).k == Reply::ERR) ++errs;
  }
  CHECK(errs > 0);
  CHECK(st.exec(V({"XREADGROUP", "GROUP", "g", "c", "BLOCK", "1", "STREAMS", "nokey", ">"})).k == Reply::ERR);
}

// ------------------------------------------------------------------ concurrent fast path
static void test_store_concurrent() {
  auto st = std::make_shared<Store>((size_t)1 << 30);
  st->exec(V({"XGROUP", "CREATE", "q", "workers", "$"}));
  const int producers = 3, per = 400;
  std::atomic<int> consumed{0}, bad{0};
  std::vector<std::thread> ts;
  for (int p = 0; p < producers; ++p)
    ts.emplace_back([&, p] {
      for (int i = 0; i < per; ++i) {
        const std::string body(16 + i % 50, (char)('a' + p));
        st->exec(V({"XADD", "q", "*", "uri", std::to_string(p) + ":" + std::to_string(i), "image", b64(body),
                    "shape", "1"}));
      }
    });
  for (int c = 0; c < 2; ++c)
    ts.emplace_back([&, c] {
      while (consumed < producers * per) {
        auto recs = st->read_batch("q", "workers", "c" + std::to_string(c), 32, 20);
        std::vector<std::string> ids;
        std::vector<std::pair<std::string, std::string>> res;
        for (auto& r : recs) {
          if (r.kind != "image" || r.payload.size() < 16) ++bad;
          ids.push_back(r.sid);
          res.emplace_back("result:" + r.uri, "ok");
        }
        st->finish("q", "workers", ids, res, "value");
        consumed += (int)recs.size();
      }
    });
  // a third connection poking at the same keys while the workers block
  ts.emplace_back([&] {
    for (int i = 0; i < 300; ++i) {
      st->exec(V({"XLEN", "q"}));
      st->exec(V({"KEYS", "result:*"}));
      st->exec(V({"INFO"}));
    }
  });
  for (auto& t : ts) t.join();
  CHECK(consumed == producers * per);
  CHECK(bad == 0);
  CHECK(st->exec(V({"XLEN", "q"})).i == 0);
  CHECK((int)st->exec(V({"KEYS", "result:*"})).a.size() == producers * per);

  // a blocked reader whose stream is deleted under it must error out, not touch freed nodes
  st->exec(V({"XGROUP", "CREATE", "gone", "g", "$"}));
  std::thread reader([&] {
    try {
      for (int i = 0; i < 50; ++i) st->read_batch("gone", "g", "c", 4, 5);
    } catch (const std::runtime_error&) {
    }
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  st->exec(V({"DEL", "gone"}));
  reader.join();
  st->shutdown();
  CHECK(st->stopping());
}

// ------------------------------------------------------------------ TCP front end
static int connect_to(int port) {
  const int fd = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  inet_pton(AF_INET, "127.0.0.1", &a.sin_addr);
  if (connect(fd, (sockaddr*)&a, sizeof(a)) != 0) {
    close(fd);
    return -1;
  }
  timeval tv{2, 0};
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  return fd;
}

static std::string roundtrip(int fd, const std::string& req, size_t want_bytes) {
  send(fd, req.data(), req.size(), MSG_NOSIGNAL);
  std::string got;
  char buf[4096];
  while (got.size() < want_bytes) {
    const ssize_t r = recv(fd, buf, sizeof(buf), 0);
    if (r <= 0) break;
    got.append(buf, (size_t)r);
  }
  return got;
}

static std::string resp(const std::vector<std::string>& a) {
  std::string o = "*" + std::to_string(a.size()) + "\r\n";
  for (auto& x : a) o += "$" + std::to_string(x.size()) + "\r\n" + x + "\r\n";
  return o;
}

static void test_server() {
  auto st = std::make_shared<Store>((size_t)1 << 30);
  Server srv(st);
  const int port = srv.start("127.0.0.1", 0);
  CHECK(port > 0);
  std::vector<std::thread> ts;
  std::atomic<int> bad{0};
  for (int c = 0; c < 4; ++c)
    ts.emplace_back([&, c] {
      const int fd = connect_to(port);
      if (fd < 0) { ++bad; return; }
      std::string req;
      for (int i = 0; i < 50; ++i) req += resp(V({"PING"}));
      const std::string pong = roundtrip(fd, req, 50 * 7);
      if (pong.size() != 50 * 7) ++bad;
      // split a command across writes: the parser must wait for the rest
      const std::string cmd = resp(V({"XADD", "tcp", "*", "uri", "c" + std::to_string(c)}));
      send(fd, cmd.data(), cmd.size() / 2, MSG_NOSIGNAL);
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
      const std::string id = roundtrip(fd, cmd.substr(cmd.size() / 2), 5);
      if (id.empty() || id[0] != '$') ++bad;
      const std::string inl = roundtrip(fd, "PING\r\n", 7);  // inline command form
      if (inl != "+PONG\r\n") ++bad;
      close(fd);
    });
  for (auto& t : ts) t.join();
  CHECK(bad == 0);
  CHECK(st->exec(V({"XLEN", "tcp"})).i == 4);

  // garbage on the wire: error reply or hang-up, the server keeps serving others
  std::mt19937 rng(5);
  for (int it = 0; it < 40; ++it) {
    const int fd = connect_to(port);
    if (fd < 0) { ++bad; continue; }
    std::string junk = "*" + std::to_string((int)(rng() % 5) - 1) + "\r\n";
    const int n = rng() % 200;
    for (int k = 0; k < n; ++k) junk.push_back((char)(rng() % 4 == 0 ? "$*\r\n"[rng() % 4] : rng()));
    junk += "\r\n";
    send(fd, junk.data(), junk.size(), MSG_NOSIGNAL);
    ::shutdown(fd, SHUT_WR);
    char buf[512];
    while (recv(fd, buf, sizeof(buf), 0) > 0) {
    }
    close(fd);
  }
  const int fd = connect_to(port);
  CHECK(fd >= 0);
  if (fd >= 0) {
    CHECK(roundtrip(fd, resp(V({"PING"})), 7) == "+PONG\r\n");
    CHECK(roundtrip(fd, resp(V({"SHUTDOWN"})), 5) == "+OK\r\n");
    close(fd);
  }
  for (int i = 0; i < 200 && srv.running(); ++i) std::this_thread::sleep_for(std::chrono::milliseconds(5));
  srv.stop();
  CHECK(!srv.running());
}

int main(int argc, char** argv) {
  const std::string only = argc > 1 ? argv[1] : "";
  struct T { const char* name; void (*fn)(); } tests[] = {
      {"crc", test_crc}, {"pb", test_pb}, {"gatherer", test_gatherer}, {"store", test_store_commands},
      {"store_concurrent", test_store_concurrent}, {"server", test_server}};
  for (auto& t : tests) {
    if (!only.empty() && only != t.name) continue;
    const int before = g_fail;
    t.fn();
    std::printf("%-18s %s\n", t.name, g_fail == before ? "ok" : "FAILED");
    std::fflush(stdout);
  }
  std::printf("rt_selftest: %s\n", g_fail ? "FAILED" : "PASSED");
  return g_fail ? 1 : 0;
}
