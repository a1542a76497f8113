// Native Cluster Serving queue: a Redis-protocol (RESP2) stream/hash store with a
// multi-threaded TCP front end and GIL-free in-process fast paths for the GPU worker.
//
// Reference: the reference's serving input/output path is a Redis server driven by a Spark
// Streaming job -- XADD to "image_stream" by the client (Py/serving/client.py:87),
// readStream(redis) micro-batches (Zs/serving/ClusterServing.scala:106-129), "result:<uri>"
// hashes written back (:276-307), memory-based trimming (:134-140). Redis is not part of
// this image, so the framework carries the subset of Redis it needs. Any RESP client
// (redis-py, redis-cli, zoo.serving.RespClient) talks to the TCP server; a worker in the
// same process skips the socket and the RESP codec: `read_batch` blocks WITHOUT the GIL,
// hands over up to `count` records with their base64 payloads already decoded (C++), and
// `finish` writes every result hash plus the XACK/XDEL of the batch under one lock.
//
// Commands: PING ECHO XADD XLEN XRANGE XGROUP CREATE/DESTROY XREADGROUP XACK XDEL XTRIM
// HSET HMSET HGET HGETALL KEYS DEL EXISTS INFO CONFIG GET/SET DBSIZE FLUSHALL SHUTDOWN.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#ifndef ZOO_RT_NO_PYTHON  // the self-test build (tools/sanitize_runtime.py) has no Python
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

namespace py = pybind11;
#endif

namespace zoo_serving {

// ------------------------------------------------------------------ replies
struct Reply {
  enum Kind { SIMPLE, ERR, INT, BULK, NIL, ARR } k = NIL;
  std::string s;
  long long i = 0;
  std::vector<Reply> a;
  static Reply simple(const std::string& v) { Reply r; r.k = SIMPLE; r.s = v; return r; }
  static Reply err(const std::string& v) { Reply r; r.k = ERR; r.s = v; return r; }
  static Reply num(long long v) { Reply r; r.k = INT; r.i = v; return r; }
  static Reply bulk(const std::string& v) { Reply r; r.k = BULK; r.s = v; return r; }
  static Reply nil() { return Reply(); }
  static Reply arr() { Reply r; r.k = ARR; return r; }
};

void encode(const Reply& r, std::string& out) {
  switch (r.k) {
    case Reply::SIMPLE: out += '+'; out += r.s; out += "\r\n"; break;
    case Reply::ERR: out += '-'; out += r.s; out += "\r\n"; break;
    case Reply::INT: out += ':'; out += std::to_string(r.i); out += "\r\n"; break;
    case Reply::NIL: out += "$-1\r\n"; break;
    case Reply::BULK:
      out += '$'; out += std::to_string(r.s.size()); out += "\r\n"; out += r.s; out += "\r\n"; break;
    case Reply::ARR:
      out += '*'; out += std::to_string(r.a.size()); out += "\r\n";
      for (const auto& x : r.a) encode(x, out);
      break;
  }
}

#ifndef ZOO_RT_NO_PYTHON
py::object to_py(const Reply& r) {
  switch (r.k) {
    case Reply::SIMPLE: return py::str(r.s);
    case Reply::ERR: throw std::runtime_error(r.s);
    case Reply::INT: return py::int_(r.i);
    case Reply::BULK: return py::bytes(r.s);
    case Reply::NIL: return py::none();
    case Reply::ARR: {
      py::list l;
      for (const auto& x : r.a) l.append(to_py(x));
      return l;
    }
  }
  return py::none();
}
#endif

// ------------------------------------------------------------------ helpers
std::string upper(std::string s) {
  for (auto& c : s) c = (char)toupper((unsigned char)c);
  return s;
}

typedef std::pair<unsigned long long, unsigned long long> Sid;

bool parse_id(const std::string& s, Sid* out) {
  const size_t d = s.find('-');
  try {
    out->first = std::stoull(s.substr(0, d));
    out->second = d == std::string::npos ? 0 : std::stoull(s.substr(d + 1));
  } catch (...) {
    return false;
  }
  return true;
}

std::string id_str(const Sid& i) { return std::to_string(i.first) + "-" + std::to_string(i.second); }

// glob match for KEYS: * ? [set] [!set] [^set] and \-escapes
bool glob(const char* p, const char* s) {
  for (; *p; ++p, ++s) {
    if (*p == '*') {
      while (p[1] == '*') ++p;
      if (!p[1]) return true;
      for (; *s; ++s)
        if (glob(p + 1, s)) return true;
      return glob(p + 1, s);
    }
    if (!*s) return false;
    if (*p == '?') continue;
    if (*p == '[') {
      const char* q = p + 1;
      bool neg = *q == '!' || *q == '^';
      if (neg) ++q;
      bool hit = false;
      for (; *q && *q != ']'; ++q) {
        if (q[1] == '-' && q[2] && q[2] != ']') {
          if (*s >= q[0] && *s <= q[2]) hit = true;
          q += 2;
        } else if (*q == *s) {
          hit = true;
        }
      }
      if (hit == neg || !*q) return false;
      p = q;
      continue;
    }
    if (*p == '\\' && p[1]) ++p;
    if (*p != *s) return false;
  }
  return !*s;
}

// base64 (RFC 4648, '=' padding, whitespace ignored)
bool b64decode(const std::string& in, std::string* out) {
  static int8_t T[256];
  static std::once_flag once;
  std::call_once(once, [] {
    memset(T, -1, sizeof(T));
    const char* a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    for (int i = 0; i < 64; ++i) T[(unsigned char)a[i]] = (int8_t)i;
    T['-'] = 62; T['_'] = 63;  // url-safe alphabet too
  });
  out->clear();
  out->reserve(in.size() / 4 * 3);
  unsigned acc = 0;
  int bits = 0;
  for (unsigned char c : in) {
    if (c == '=') break;
    if (c == '\n' || c == '\r' || c == ' ' || c == '\t') continue;
    const int v = T[c];
    if (v < 0) return false;
    acc = (acc << 6) | (unsigned)v;
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out->push_back((char)((acc >> bits) & 0xff));
    }
  }
  return true;
}

// ------------------------------------------------------------------ store
typedef std::vector<std::pair<std::string, std::string>> Fields;

struct Entry {
  Fields f;
  size_t size = 0;
};

struct Group {
  Sid last{0, 0};
  std::unordered_map<std::string, std::string> pending;  // id -> consumer
};

struct Stream {
  std::map<Sid, Entry> e;
  Sid last{0, 0};
  std::map<std::string, Group> groups;
};

typedef std::unordered_map<std::string, std::string> Hash;

// Key space split over 64 hash tables. One std::unordered_map holding every result key rehashes
// all of it when it doubles: at a few 100k keys that is a 20-100 ms stop of the whole store under
// its lock (every XADD, read and finish waits), which was the latency tail of the open-loop
// serving bench (profiles/r6/serving.md). With 64 shards each doubling moves 1/64 of the keys.
template <class V>
class ShardedMap {
 public:
  static constexpr int kShards = 64;
  ShardedMap() {
    for (auto& s : s_) s.reserve(1024);
  }
  V* find(const std::string& k) {
    auto& s = shard(k);
    auto it = s.find(k);
    return it == s.end() ? nullptr : &it->second;
  }
  V& operator[](const std::string& k) { return shard(k)[k]; }
  size_t count(const std::string& k) const { return shard(k).count(k); }
  size_t erase(const std::string& k) { return shard(k).erase(k); }
  size_t size() const {
    size_t n = 0;
    for (auto& s : s_) n += s.size();
    return n;
  }
  void clear() {
    for (auto& s : s_) s.clear();
  }
  template <class F>
  void for_each(F&& f) const {
    for (auto& s : s_)
      for (auto& kv : s) f(kv.first, kv.second);
  }

 private:
  std::unordered_map<std::string, V>& shard(const std::string& k) { return s_[pick(k)]; }
  const std::unordered_map<std::string, V>& shard(const std::string& k) const { return s_[pick(k)]; }
  // the top bits pick the shard; the table inside buckets by the value modulo its size
  static size_t pick(const std::string& k) { return (std::hash<std::string>()(k) >> 58) & (kShards - 1); }
  std::unordered_map<std::string, V> s_[kShards];
};

struct Record {
  std::string sid, uri, kind, payload, shape;
};

class Store {
 public:
  explicit Store(size_t maxmem) : maxmem_(maxmem) {}

  Reply exec(const std::vector<std::string>& a) {
    if (a.empty()) return Reply::err("ERR empty command");
    const std::string cmd = upper(a[0]);
    try {
      if (cmd == "XREADGROUP") return xreadgroup(a);  // manages the lock itself (may block)
      std::lock_guard<std::mutex> g(mu_);
      return dispatch(cmd, a);
    } catch (const std::exception& e) {
      return Reply::err(std::string("ERR ") + e.what());
    }
  }

  // fast path: up to `count` new records for (group, consumer), base64 payloads decoded
  std::vector<Record> read_batch(const std::string& key, const std::string& group, const std::string& consumer,
                                 int count, int block_ms) {
    std::vector<Record> out;
    std::vector<std::pair<std::string, Fields>> got;
    {
      std::unique_lock<std::mutex> lk(mu_);
      const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(block_ms > 0 ? block_ms : 0);
      bool last = false;
      while (true) {
        // look the stream up again after every wait: a DEL / FLUSHALL / XGROUP DESTROY from
        // another connection may have erased it while the lock was released
        auto it = streams_.find(key);
        if (it == streams_.end() || !it->second.groups.count(group)) throw std::runtime_error("NOGROUP No such key or consumer group");
        take(it->second, it->second.groups[group], consumer, count, &got);
        if (last || !got.empty() || block_ms <= 0 || stop_) break;
        last = cv_.wait_until(lk, deadline) == std::cv_status::timeout;
      }
    }
    for (auto& m : got) {
      Record r;
      r.sid = m.first;
      const std::string* img = nullptr;
      const std::string* ten = nullptr;
      for (auto& kv : m.second) {
        if (kv.first == "uri") r.uri = kv.second;
        else if (kv.first == "image") img = &kv.second;
        else if (kv.first == "tensor") ten = &kv.second;
        else if (kv.first == "shape") r.shape = kv.second;
      }
      if (img) r.kind = "image";
      else if (ten) r.kind = "tensor";
      if ((img || ten) && !b64decode(img ? *img : *ten, &r.payload)) r.kind = "bad";
      out.push_back(std::move(r));
    }
    return out;
  }

  // latency tracking for the load generator: finish() stamps every result key it writes
  void track(bool on) {
    std::lock_guard<std::mutex> g(mu_);
    track_ = on;
    done_.clear();
  }
  // completion stamps (steady-clock ns, -1 = not finished) of keys[idx[j]] -> (*out)[idx[j]]; the
  // lock is taken per 256 keys so a poll over 100k keys never holds the serving worker's finish()
  void done_times(const std::vector<std::string>& keys, const std::vector<size_t>& idx,
                  std::vector<long long>* out) {
    out->resize(keys.size(), -1);
    for (size_t j0 = 0; j0 < idx.size(); j0 += 256) {
      std::lock_guard<std::mutex> g(mu_);
      for (size_t j = j0; j < std::min(idx.size(), j0 + 256); ++j) {
        const long long* d = done_.find(keys[idx[j]]);
        (*out)[idx[j]] = d == nullptr ? -1 : *d;
      }
    }
  }

  // fast path: HSET key field value for every result, then XACK + XDEL the ids
  void finish(const std::string& key, const std::string& group, const std::vector<std::string>& ids,
              const std::vector<std::pair<std::string, std::string>>& results, const std::string& field) {
    std::lock_guard<std::mutex> g(mu_);
    if (track_) {
      const long long now = std::chrono::duration_cast<std::chrono::nanoseconds>(
                                std::chrono::steady_clock::now().time_since_epoch()).count();
      for (auto& r : results) done_[r.first] = now;
    }
    for (auto& r : results) {
      if (streams_.count(r.first)) continue;
      auto& h = hashes_[r.first];
      auto it = h.find(field);
      if (it != h.end()) used_ -= field.size() + it->second.size();
      used_ += field.size() + r.second.size();
      h[field] = r.second;
    }
    auto it = streams_.find(key);
    if (it != streams_.end()) {
      auto gi = it->second.groups.find(group);
      for (auto& id : ids) {
        if (gi != it->second.groups.end()) gi->second.pending.erase(id);
        Sid s;
        if (parse_id(id, &s)) {
          auto e = it->second.e.find(s);
          if (e != it->second.e.end()) {
            used_ -= e->second.size;
            it->second.e.erase(e);
          }
        }
      }
    }
    cv_.notify_all();
  }

  void shutdown() {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
    cv_.notify_all();
  }
  bool stopping() {
    std::lock_guard<std::mutex> g(mu_);
    return stop_;
  }

 private:
  static size_t fsize(const Fields& f) {
    size_t n = 64;
    for (auto& kv : f) n += kv.first.size() + kv.second.size();
    return n;
  }

  void take(Stream& s, Group& g, const std::string& consumer, int count,
            std::vector<std::pair<std::string, Fields>>* got) {
    for (auto it = s.e.upper_bound(g.last); it != s.e.end() && (count <= 0 || (int)got->size() < count); ++it) {
      const std::string sid = id_str(it->first);
      g.last = it->first;
      g.pending[sid] = consumer;
      got->push_back({sid, it->second.f});
    }
  }

  bool wrong_type_stream(const std::string& k) { return hashes_.count(k) > 0; }
  bool wrong_type_hash(const std::string& k) { return streams_.count(k) > 0; }

  Reply entry_list(const std::map<Sid, Entry>::const_iterator& it) {
    Reply one = Reply::arr();
    one.a.push_back(Reply::bulk(id_str(it->first)));
    Reply kv = Reply::arr();
    for (auto& f : it->second.f) {
      kv.a.push_back(Reply::bulk(f.first));
      kv.a.push_back(Reply::bulk(f.second));
    }
    one.a.push_back(kv);
    return one;
  }

  size_t trim(Stream& s, size_t maxlen) {
    size_t n = 0;
    while (s.e.size() > maxlen) {
      used_ -= s.e.begin()->second.size;
      s.e.erase(s.e.begin());
      ++n;
    }
    return n;
  }

  Reply dispatch(const std::string& cmd, const std::vector<std::string>& a) {
    const size_t n = a.size();
    if (cmd == "PING") return n > 1 ? Reply::bulk(a[1]) : Reply::simple("PONG");
    if (cmd == "ECHO") return Reply::bulk(a.at(1));
    if (cmd == "DBSIZE") return Reply::num((long long)(streams_.size() + hashes_.size()));
    if (cmd == "FLUSHALL" || cmd == "FLUSHDB") {
      streams_.clear();
      hashes_.clear();
      used_ = 0;
      return Reply::simple("OK");
    }
    if (cmd == "INFO") {
      return Reply::bulk("# Memory\r\nused_memory:" + std::to_string(used_) + "\r\nmaxmemory:" +
                         std::to_string(maxmem_) + "\r\n# Keyspace\r\ndb0:keys=" +
                         std::to_string(streams_.size() + hashes_.size()) + "\r\n");
    }
    if (cmd == "CONFIG") {
      const std::string sub = upper(a.at(1));
      if (sub == "SET" && n >= 4 && upper(a[2]) == "MAXMEMORY") {
        std::string v = a[3];
        double mult = 1;
        const char last = (char)tolower(v.back());
        if (last == 'k' || last == 'm' || last == 'g') {
          mult = last == 'k' ? 1024.0 : last == 'm' ? 1048576.0 : 1073741824.0;
          v.pop_back();
        }
        maxmem_ = (size_t)(std::stod(v) * mult);
        return Reply::simple("OK");
      }
      if (sub == "GET") {
        Reply r = Reply::arr();
        r.a.push_back(Reply::bulk("maxmemory"));
        r.a.push_back(Reply::bulk(std::to_string(maxmem_)));
        return r;
      }
      return Reply::simple("OK");
    }
    if (cmd == "XADD") {
      size_t i = 2;
      long long maxlen = -1;
      if (upper(a.at(i)) == "MAXLEN") {
        ++i;
        if (a.at(i) == "~" || a[i] == "=") ++i;
        maxlen = std::stoll(a.at(i++));
      }
      const std::string rid = a.at(i++);
      if ((n - i) % 2 || n == i) return Reply::err("ERR wrong number of arguments for 'xadd' command");
      if (wrong_type_stream(a[1])) return Reply::err("WRONGTYPE Operation against a key holding the wrong kind of value");
      Entry e;
      for (; i < n; i += 2) e.f.push_back({a[i], a[i + 1]});
      e.size = fsize(e.f);
      if (used_ + e.size > maxmem_) return Reply::err("OOM command not allowed when used memory > 'maxmemory'.");
      Stream& s = streams_[a[1]];
      Sid nid;
      if (rid == "*") {
        const unsigned long long ms = (unsigned long long)std::chrono::duration_cast<std::chrono::milliseconds>(
                                          std::chrono::system_clock::now().time_since_epoch()).count();
        nid = ms > s.last.first ? Sid{ms, 0} : Sid{s.last.first, s.last.second + 1};
      } else {
        if (!parse_id(rid, &nid)) return Reply::err("ERR Invalid stream ID specified as stream command argument");
        if (nid <= s.last)
          return Reply::err("ERR The ID specified in XADD is equal or smaller than the target stream top item");
      }
      s.last = nid;
      used_ += e.size;
      s.e.emplace(nid, std::move(e));
      if (maxlen >= 0) trim(s, (size_t)maxlen);
      cv_.notify_all();
      return Reply::bulk(id_str(nid));
    }
    if (cmd == "XLEN") {
      auto it = streams_.find(a.at(1));
      return Reply::num(it == streams_.end() ? 0 : (long long)it->second.e.size());
    }
    if (cmd == "XTRIM") {
      auto it = streams_.find(a.at(1));
      size_t i = 3;
      if (a.at(i) == "~" || a[i] == "=") ++i;
      return Reply::num(it == streams_.end() ? 0 : (long long)trim(it->second, std::stoull(a.at(i))));
    }
    if (cmd == "XRANGE") {
      Reply r = Reply::arr();
      auto it = streams_.find(a.at(1));
      if (it == streams_.end()) return r;
      Sid lo{0, 0}, hi{~0ull, ~0ull};
      if (a.at(2) != "-" && !parse_id(a[2], &lo)) return Reply::err("ERR Invalid stream ID");
      if (a.at(3) != "+" && !parse_id(a[3], &hi)) return Reply::err("ERR Invalid stream ID");
      long long cnt = -1;
      if (n >= 6 && upper(a[4]) == "COUNT") cnt = std::stoll(a[5]);
      for (auto e = it->second.e.lower_bound(lo); e != it->second.e.end() && e->first <= hi; ++e) {
        if (cnt >= 0 && (long long)r.a.size() >= cnt) break;
        r.a.push_back(entry_list(e));
      }
      return r;
    }
    if (cmd == "XGROUP") {
      const std::string sub = upper(a.at(1));
      if (sub == "CREATE") {
        if (wrong_type_stream(a.at(2))) return Reply::err("WRONGTYPE Operation against a key holding the wrong kind of value");
        Stream& s = streams_[a[2]];
        if (s.groups.count(a.at(3))) return Reply::err("BUSYGROUP Consumer Group name already exists");
        Group g;
        const std::string& start = a.at(4);
        if (start == "$") g.last = s.last;
        else if (!parse_id(start, &g.last)) return Reply::err("ERR Invalid stream ID");
        s.groups[a[3]] = g;
        return Reply::simple("OK");
      }
      if (sub == "DESTROY") {
        auto it = streams_.find(a.at(2));
        return Reply::num(it != streams_.end() && it->second.groups.erase(a.at(3)) ? 1 : 0);
      }
      return Reply::err("ERR unsupported XGROUP subcommand");
    }
    if (cmd == "XACK") {
      auto it = streams_.find(a.at(1));
      if (it == streams_.end()) return Reply::num(0);
      auto g = it->second.groups.find(a.at(2));
      if (g == it->second.groups.end()) return Reply::num(0);
      long long c = 0;
      for (size_t i = 3; i < n; ++i) c += (long long)g->second.pending.erase(a[i]);
      return Reply::num(c);
    }
    if (cmd == "XDEL") {
      auto it = streams_.find(a.at(1));
      if (it == streams_.end()) return Reply::num(0);
      long long c = 0;
      for (size_t i = 2; i < n; ++i) {
        Sid s;
        if (!parse_id(a[i], &s)) continue;
        auto e = it->second.e.find(s);
        if (e != it->second.e.end()) {
          used_ -= e->second.size;
          it->second.e.erase(e);
          ++c;
        }
      }
      return Reply::num(c);
    }
    if (cmd == "HSET" || cmd == "HMSET") {
      if (n < 4 || (n - 2) % 2) return Reply::err("ERR wrong number of arguments for 'hset' command");
      if (wrong_type_hash(a[1])) return Reply::err("WRONGTYPE Operation against a key holding the wrong kind of value");
      auto& h = hashes_[a[1]];
      long long added = 0;
      for (size_t i = 2; i < n; i += 2) {
        auto it = h.find(a[i]);
        if (it == h.end()) ++added;
        else used_ -= a[i].size() + it->second.size();
        used_ += a[i].size() + a[i + 1].size();
        h[a[i]] = a[i + 1];
      }
      cv_.notify_all();
      return cmd == "HMSET" ? Reply::simple("OK") : Reply::num(added);
    }
    if (cmd == "HGET") {
      const Hash* h = hashes_.find(a.at(1));
      if (h == nullptr) return Reply::nil();
      auto f = h->find(a.at(2));
      return f == h->end() ? Reply::nil() : Reply::bulk(f->second);
    }
    if (cmd == "HGETALL") {
      Reply r = Reply::arr();
      const Hash* h = hashes_.find(a.at(1));
      if (h == nullptr) return r;
      for (auto& kv : *h) {
        r.a.push_back(Reply::bulk(kv.first));
        r.a.push_back(Reply::bulk(kv.second));
      }
      return r;
    }
    if (cmd == "KEYS") {
      Reply r = Reply::arr();
      const std::string& pat = a.at(1);
      for (auto& kv : streams_)
        if (glob(pat.c_str(), kv.first.c_str())) r.a.push_back(Reply::bulk(kv.first));
      hashes_.for_each([&](const std::string& k, const Hash&) {
        if (glob(pat.c_str(), k.c_str())) r.a.push_back(Reply::bulk(k));
      });
      return r;
    }
    if (cmd == "EXISTS") {
      long long c = 0;
      for (size_t i = 1; i < n; ++i) c += (streams_.count(a[i]) || hashes_.count(a[i])) ? 1 : 0;
      return Reply::num(c);
    }
    if (cmd == "DEL") {
      long long c = 0;
      for (size_t i = 1; i < n; ++i) {
        const Hash* h = hashes_.find(a[i]);
        if (h != nullptr) {
          for (auto& kv : *h) used_ -= kv.first.size() + kv.second.size();
          hashes_.erase(a[i]);
          ++c;
          continue;
        }
        auto s = streams_.find(a[i]);
        if (s != streams_.end()) {
          for (auto& e : s->second.e) used_ -= e.second.size;
          streams_.erase(s);
          ++c;
        }
      }
      return Reply::num(c);
    }
    return Reply::err("ERR unknown command '" + cmd + "'");
  }

  Reply xreadgroup(const std::vector<std::string>& a) {
    size_t i = 1;
    if (upper(a.at(i++)) != "GROUP") return Reply::err("ERR syntax error");
    const std::string group = a.at(i++), consumer = a.at(i++);
    int count = 0;
    long long block = -1;
    while (i < a.size()) {
      const std::string o = upper(a[i]);
      if (o == "COUNT") { count = std::stoi(a.at(i + 1)); i += 2; }
      else if (o == "BLOCK") { block = std::stoll(a.at(i + 1)); i += 2; }
      else if (o == "NOACK") { ++i; }
      else break;
    }
    if (i >= a.size() || upper(a[i++]) != "STREAMS") return Reply::err("ERR syntax error");
    const size_t half = (a.size() - i) / 2;
    std::unique_lock<std::mutex> lk(mu_);
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(block > 0 ? block : 0);
    while (true) {
      Reply res = Reply::arr();
      for (size_t k = 0; k < half; ++k) {
        const std::string& key = a[i + k];
        auto it = streams_.find(key);
        if (it == streams_.end() || !it->second.groups.count(group))
          return Reply::err("NOGROUP No such key or consumer group");
        if (a[i + half + k] != ">") continue;
        std::vector<std::pair<std::string, Fields>> got;
        take(it->second, it->second.groups[group], consumer, count, &got);
        if (got.empty()) continue;
        Reply sr = Reply::arr();
        sr.a.push_back(Reply::bulk(key));
        Reply msgs = Reply::arr();
        for (auto& m : got) {
          Reply one = Reply::arr();
          one.a.push_back(Reply::bulk(m.first));
          Reply kv = Reply::arr();
          for (auto& f : m.second) {
            kv.a.push_back(Reply::bulk(f.first));
            kv.a.push_back(Reply::bulk(f.second));
          }
          one.a.push_back(kv);
          msgs.a.push_back(one);
        }
        sr.a.push_back(msgs);
        res.a.push_back(sr);
      }
      if (!res.a.empty()) return res;
      if (block < 0 || stop_) return Reply::nil();
      if (block == 0) cv_.wait(lk);
      else if (cv_.wait_until(lk, deadline) == std::cv_status::timeout) block = -1;  // one last look, then nil
    }
  }

  std::mutex mu_;
  std::condition_variable cv_;
  std::unordered_map<std::string, Stream> streams_;
  ShardedMap<Hash> hashes_;
  size_t used_ = 0, maxmem_;
  bool stop_ = false;
  bool track_ = false;
  ShardedMap<long long> done_;  // result key -> finish stamp (ns)
};

// ------------------------------------------------------------------ TCP front end
class Server {
 public:
  explicit Server(std::shared_ptr<Store> st) : store_(std::move(st)) {}
  ~Server() {
    stop();
    std::lock_guard<std::mutex> g(cmu_);
    if (stopper_.joinable()) stopper_.join();
  }

  int start(const std::string& host, int port) {
    lfd_ = socket(AF_INET, SOCK_STREAM, 0);
    if (lfd_ < 0) throw std::runtime_error("socket() failed");
    int one = 1;
    setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in addr{};
    addr.sin_family = AF_INET;
    addr.sin_port = htons((uint16_t)port);
    if (inet_pton(AF_INET, host.c_str(), &addr.sin_addr) != 1) throw std::runtime_error("bad host " + host);
    if (bind(lfd_, (sockaddr*)&addr, sizeof(addr)) != 0) {
      close(lfd_);
      throw std::runtime_error("bind failed on " + host + ":" + std::to_string(port));
    }
    listen(lfd_, 128);
    socklen_t len = sizeof(addr);
    getsockname(lfd_, (sockaddr*)&addr, &len);
    port_ = ntohs(addr.sin_port);
    running_ = true;
    acceptor_ = std::thread([this] { accept_loop(); });
    return port_;
  }

  // idempotent; a second caller blocks until the first one has joined every thread, so
  // the Server can be destroyed as soon as any stop() returns
  void stop() {
    std::lock_guard<std::mutex> sg(stop_mu_);
    if (!running_.exchange(false)) return;
    store_->shutdown();
    ::shutdown(lfd_, SHUT_RDWR);
    close(lfd_);
    if (acceptor_.joinable()) acceptor_.join();
    std::vector<std::thread> ts;
    {
      std::lock_guard<std::mutex> g(cmu_);
      for (int fd : conns_) ::shutdown(fd, SHUT_RDWR);
      ts.swap(threads_);
    }
    for (auto& t : ts)
      if (t.joinable()) t.join();
  }

  int port() const { return port_; }
  bool running() const { return running_; }

 private:
  void accept_loop() {
    while (running_) {
      const int fd = accept(lfd_, nullptr, nullptr);
      if (fd < 0) {
        if (!running_) break;
        continue;
      }
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      std::lock_guard<std::mutex> g(cmu_);
      conns_.insert(fd);
      threads_.emplace_back([this, fd] { serve(fd); });
    }
  }

  // parse one RESP command from buf[pos..]; returns false if incomplete
  static bool parse(const std::string& buf, size_t* pos, std::vector<std::string>* args) {
    size_t p = *pos;
    args->clear();
    auto line = [&](size_t from, size_t* eol) {
      const size_t e = buf.find("\r\n", from);
      if (e == std::string::npos) return false;
      *eol = e;
      return true;
    };
    size_t e;
    if (p >= buf.size()) return false;
    if (buf[p] != '*') {  // inline command
      if (!line(p, &e)) return false;
      std::string l = buf.substr(p, e - p);
      size_t s = 0;
      while (s < l.size()) {
        while (s < l.size() && l[s] == ' ') ++s;
        size_t t = l.find(' ', s);
        if (t == std::string::npos) t = l.size();
        if (t > s) args->push_back(l.substr(s, t - s));
        s = t;
      }
      *pos = e + 2;
      return true;
    }
    if (!line(p, &e)) return false;
    const long cnt = std::stol(buf.substr(p + 1, e - p - 1));
    p = e + 2;
    for (long i = 0; i < cnt; ++i) {
      if (p >= buf.size() || !line(p, &e)) return false;
      if (buf[p] != '$') throw std::runtime_error("protocol error: expected bulk string");
      const long n = std::stol(buf.substr(p + 1, e - p - 1));
      p = e + 2;
      if (n < 0) { args->push_back(""); continue; }
      if (buf.size() < p + (size_t)n + 2) return false;
      args->push_back(buf.substr(p, (size_t)n));
      p += (size_t)n + 2;
    }
    *pos = p;
    return true;
  }

  void serve(int fd) {
    std::string buf, out;
    std::vector<std::string> args;
    char tmp[1 << 16];
    bool alive = true, shutdown_req = false;
    while (alive && running_) {
      const ssize_t r = recv(fd, tmp, sizeof(tmp), 0);
      if (r <= 0) break;
      buf.append(tmp, (size_t)r);
      size_t pos = 0;
      out.clear();
      try {
        while (parse(buf, &pos, &args)) {
          if (args.empty()) continue;
          if (upper(args[0]) == "SHUTDOWN") {
            out += "+OK\r\n";
            alive = false;
            shutdown_req = true;
            break;
          }
          encode(store_->exec(args), out);
        }
      } catch (const std::exception& ex) {
        out += std::string("-ERR ") + ex.what() + "\r\n";
        alive = false;
      }
      buf.erase(0, pos);
      size_t off = 0;
      while (off < out.size()) {
        const ssize_t w = send(fd, out.data() + off, out.size() - off, MSG_NOSIGNAL);
        if (w <= 0) { alive = false; break; }
        off += (size_t)w;
      }
    }
    {
      std::lock_guard<std::mutex> g(cmu_);
      conns_.erase(fd);
      // SHUTDOWN: stop from a separate (joined) thread, after the +OK went out -- stop()
      // joins this connection thread, so it cannot run here
      if (shutdown_req && !stopper_.joinable()) stopper_ = std::thread([this] { stop(); });
    }
    close(fd);
  }

  std::shared_ptr<Store> store_;
  int lfd_ = -1, port_ = 0;
  std::atomic<bool> running_{false};
  std::thread acceptor_;
  std::mutex cmu_, stop_mu_;
  std::set<int> conns_;
  std::vector<std::thread> threads_;
  std::thread stopper_;
};

// ------------------------------------------------------------------ load generator
// Open-loop client for Cluster Serving measurements (BASELINE config 5): `threads` C++ threads
// send records on a fixed schedule (record i is due at t0 + i / rate, whatever the responses)
// for `duration` seconds, either straight into the in-process store (XADD through exec, the
// path a co-located producer takes) or over TCP/RESP to the server's port (the network path of
// the reference client, Py/serving/client.py:25-150). Completion is the store's finish() stamp
// of the record's result key; latency = stamp - send time, both on this process's steady clock.
// Replaces Python client processes, which saturated at ~6-8k records/s on the box's CPUs.
struct LoadGenStats {
  long long sent = 0, measured = 0, completed = 0, unfinished = 0;
  double offered = 0, achieved = 0, p50 = 0, p90 = 0, p99 = 0, mean = 0, max = 0;
};

static long long lg_now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

static void lg_resp_cmd(const std::vector<const std::string*>& parts, std::string& out) {
  out += '*';
  out += std::to_string(parts.size());
  out += "\r\n";
  for (auto* p : parts) {
    out += '$';
    out += std::to_string(p->size());
    out += "\r\n";
    out += *p;
    out += "\r\n";
  }
}

// read exactly one RESP reply line-group for an XADD (a bulk string or an error line)
static bool lg_read_reply(int fd, std::string& buf) {
  while (true) {
    const size_t nl = buf.find("\r\n");
    if (nl != std::string::npos) {
      if (buf[0] == '$') {
        const long len = std::strtol(buf.c_str() + 1, nullptr, 10);
        const size_t need = nl + 2 + (len > 0 ? (size_t)len + 2 : 0);
        if (buf.size() >= need) {
          buf.erase(0, need);
          return true;
        }
      } else {
        buf.erase(0, nl + 2);
        return true;
      }
    }
    char tmp[4096];
    const ssize_t r = ::recv(fd, tmp, sizeof(tmp), 0);
    if (r <= 0) return false;
    buf.append(tmp, (size_t)r);
  }
}

LoadGenStats run_loadgen(const std::shared_ptr<Store>& st, const std::string& stream, const std::string& kind,
                         const std::vector<std::string>& payloads, const std::string& shape, double rate,
                         double duration, int threads, const std::string& prefix, double warm, double grace,
                         int tcp_port) {
  LoadGenStats S;
  const long long n = (long long)(rate * duration);
  if (n <= 0 || payloads.empty()) return S;
  if (threads < 1) threads = 1;
  std::vector<long long> sent_ns((size_t)n, -1);
  std::vector<std::string> keys((size_t)n);
  for (long long i = 0; i < n; ++i) keys[(size_t)i] = "result:" + prefix + "-" + std::to_string(i);
  const std::string xadd = "XADD", star = "*", f_uri = "uri", f_shape = "shape";
  const long long t0 = lg_now_ns() + 20000000LL;  // 20 ms for the threads to start
  const double step_ns = 1e9 / rate;
  std::atomic<long long> errors{0};
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t) {
    th.emplace_back([&, t] {
      int fd = -1;
      std::string rbuf, wbuf;
      if (tcp_port > 0) {
        fd = ::socket(AF_INET, SOCK_STREAM, 0);
        sockaddr_in a{};
        a.sin_family = AF_INET;
        a.sin_port = htons((uint16_t)tcp_port);
        a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
        int one = 1;
        ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        if (::connect(fd, (sockaddr*)&a, sizeof(a)) != 0) {
          ::close(fd);
          errors += 1;
          return;
        }
      }
      for (long long i = t; i < n; i += threads) {
        const long long due = t0 + (long long)(i * step_ns);
        std::this_thread::sleep_until(std::chrono::steady_clock::time_point(std::chrono::nanoseconds(due)));
        const std::string uri = prefix + "-" + std::to_string(i);
        const std::string& pl = payloads[(size_t)(i % (long long)payloads.size())];
        sent_ns[(size_t)i] = lg_now_ns();
        if (fd >= 0) {
          wbuf.clear();
          std::vector<const std::string*> parts{&xadd, &stream, &star, &f_uri, &uri, &kind, &pl};
          if (!shape.empty()) { parts.push_back(&f_shape); parts.push_back(&shape); }
          lg_resp_cmd(parts, wbuf);
          size_t off = 0;
          while (off < wbuf.size()) {
            const ssize_t w = ::send(fd, wbuf.data() + off, wbuf.size() - off, MSG_NOSIGNAL);
            if (w <= 0) break;
            off += (size_t)w;
          }
          if (off < wbuf.size() || !lg_read_reply(fd, rbuf)) {
            errors += 1;
            break;
          }
        } else {
          std::vector<std::string> cmd{xadd, stream, star, f_uri, uri, kind, pl};
          if (!shape.empty()) { cmd.push_back(f_shape); cmd.push_back(shape); }
          const Reply r = st->exec(cmd);
          if (r.k == Reply::ERR) errors += 1;
        }
      }
      if (fd >= 0) ::close(fd);
    });
  }
  for (auto& x : th) x.join();
  // wait for the tail (or the grace period)
  std::vector<long long> done((size_t)n, -1);
  std::vector<size_t> left;
  for (long long i = 0; i < n; ++i)
    if (sent_ns[(size_t)i] >= 0) left.push_back((size_t)i);
  const long long deadline = lg_now_ns() + (long long)(grace * 1e9);
  while (true) {
    st->done_times(keys, left, &done);   // only the keys still open
    size_t k = 0;
    for (size_t i : left)
      if (done[i] < 0) left[k++] = i;
    left.resize(k);
    if (left.empty() || lg_now_ns() > deadline) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  const long long w0 = t0 + (long long)(warm * 1e9), w1 = t0 + (long long)(duration * 1e9);
  std::vector<double> lat;
  long long fin_in_window = 0;
  for (long long i = 0; i < n; ++i) {
    const long long s0 = sent_ns[(size_t)i], d = done[(size_t)i];
    if (s0 < 0) continue;
    ++S.sent;
    if (d < 0) ++S.unfinished;
    if (d >= w0 && d <= w1) ++fin_in_window;
    if (s0 >= w0 && s0 <= w1) {
      ++S.measured;
      if (d >= 0) lat.push_back((d - s0) * 1e-6);
    }
  }
  S.completed = (long long)lat.size();
  S.offered = S.sent / duration;
  S.achieved = fin_in_window / std::max(1e-9, duration - warm);
  if (!lat.empty()) {
    std::sort(lat.begin(), lat.end());
    auto pct = [&](double q) { return lat[std::min(lat.size() - 1, (size_t)(q / 100.0 * (lat.size() - 1) + 0.5))]; };
    S.p50 = pct(50);
    S.p90 = pct(90);
    S.p99 = pct(99);
    S.max = lat.back();
    double sum = 0;
    for (double v : lat) sum += v;
    S.mean = sum / lat.size();
  }
  if (errors.load() > 0) S.unfinished += errors.load();
  return S;
}

// ------------------------------------------------------------------ python facade
#ifndef ZOO_RT_NO_PYTHON
class NativeStore {
 public:
  explicit NativeStore(size_t maxmem) : store_(std::make_shared<Store>(maxmem)) {}
  ~NativeStore() {
    if (server_) server_->stop();
  }

  py::object execute(const std::vector<std::string>& args) {
    Reply r;
    {
      py::gil_scoped_release nogil;
      r = store_->exec(args);
    }
    return to_py(r);
  }

  int serve(const std::string& host, int port) {
    if (server_ && server_->running()) return server_->port();
    server_ = std::make_unique<Server>(store_);
    return server_->start(host, port);
  }

  void stop() {
    if (server_) {
      py::gil_scoped_release nogil;
      server_->stop();
    }
  }

  bool running() const { return server_ && server_->running(); }

  py::list read_batch(const std::string& key, const std::string& group, const std::string& consumer, int count,
                      int block_ms) {
    std::vector<Record> recs;
    {
      py::gil_scoped_release nogil;
      recs = store_->read_batch(key, group, consumer, count, block_ms);
    }
    py::list out;
    for (auto& r : recs)
      out.append(py::make_tuple(py::bytes(r.sid), py::str(r.uri), py::str(r.kind), py::bytes(r.payload),
                                py::str(r.shape)));
    return out;
  }

  void finish(const std::string& key, const std::string& group, const std::vector<std::string>& ids,
              const std::vector<std::pair<std::string, std::string>>& results, const std::string& field) {
    py::gil_scoped_release nogil;
    store_->finish(key, group, ids, results, field);
  }

  void track(bool on) { store_->track(on); }

  // open-loop load generator (run_loadgen); blocks without the GIL, returns the measurement
  py::dict loadgen(const std::string& stream, const std::string& kind, const std::vector<std::string>& payloads,
                   const std::string& shape, double rate, double duration, int threads, const std::string& prefix,
                   double warm, double grace, bool tcp) {
    LoadGenStats S;
    const int port = tcp && server_ && server_->running() ? server_->port() : 0;
    if (tcp && port == 0) throw std::runtime_error("loadgen over TCP needs a running server (serve())");
    {
      py::gil_scoped_release nogil;
      S = run_loadgen(store_, stream, kind, payloads, shape, rate, duration, threads, prefix, warm, grace, port);
    }
    py::dict d;
    d["sent"] = S.sent; d["measured"] = S.measured; d["completed"] = S.completed; d["unfinished"] = S.unfinished;
    d["offered_rate"] = S.offered; d["achieved_throughput"] = S.achieved;
    d["p50_ms"] = S.p50; d["p90_ms"] = S.p90; d["p99_ms"] = S.p99; d["mean_ms"] = S.mean; d["max_ms"] = S.max;
    return d;
  }

 private:
  std::shared_ptr<Store> store_;
  std::unique_ptr<Server> server_;
};
#endif  // ZOO_RT_NO_PYTHON

}  // namespace zoo_serving

#ifndef ZOO_RT_NO_PYTHON

void register_serving(py::module& m) {
  using zoo_serving::NativeStore;
  py::class_<NativeStore>(m, "NativeStore")
      .def(py::init<size_t>(), py::arg("maxmemory") = (size_t)4 << 30)
      .def("execute", &NativeStore::execute)
      .def("serve", &NativeStore::serve)
      .def("stop", &NativeStore::stop)
      .def("running", &NativeStore::running)
      .def("read_batch", &NativeStore::read_batch)
      .def("finish", &NativeStore::finish)
      .def("track", &NativeStore::track, "stamp every result key finish() writes (load-generator latency)")
      .def("loadgen", &NativeStore::loadgen, py::arg("stream"), py::arg("kind"), py::arg("payloads"),
           py::arg("shape") = "", py::arg("rate") = 1000.0, py::arg("duration") = 5.0, py::arg("threads") = 4,
           py::arg("prefix") = "lg", py::arg("warm") = 1.0, py::arg("grace") = 10.0, py::arg("tcp") = false,
           "open-loop C++ load generator: records on a fixed schedule (in-process XADD or RESP over TCP), "
           "latency from the store's finish stamps; returns offered/achieved rates and p50/p90/p99");
  m.def("b64decode", [](const std::string& s) {
    std::string out;
    if (!zoo_serving::b64decode(s, &out)) throw std::runtime_error("invalid base64");
    return py::bytes(out);
  });
}
#endif  // ZOO_RT_NO_PYTHON
