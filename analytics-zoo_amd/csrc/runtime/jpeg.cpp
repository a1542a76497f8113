// Baseline / extended-sequential Huffman JPEG entropy decoder (host side of the GPU JPEG path).
//
// Serving decodes every request image before the model sees it (PreProcessing.scala:24-53 in
// the reference, OpenCV imdecode per record on the JVM). Here the work is split the MI355X way:
// the CPU does only what is inherently serial -- marker parsing and the Huffman bit-stream --
// on a C++ thread pool with the GIL released, and emits the quantised DCT coefficients of
// every 8x8 block (natural order, int16) plus the quantisation tables; dequantisation, the
// 8x8 IDCT, chroma upsampling, YCbCr->RGB and the resize / normalise to the model input all
// run as HIP kernels (csrc/kernels/image.hip) on the whole batch at once.
//
// Supported: SOF0 / SOF1 (8-bit), 1 or 3 components, any sampling factors 1..2, restart
// intervals, interleaved and non-interleaved scans. Progressive (SOF2), arithmetic coding,
// 12-bit and lossless streams return an error code and the caller falls back to the CPU
// decoder.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace zoo_jpeg {

enum Err { OK = 0, E_TRUNC = 1, E_MARKER = 2, E_UNSUPPORTED = 3, E_HUFF = 4, E_TABLE = 5, E_GEOM = 6 };

static const uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Huff {
  // canonical decode tables: maxcode / valptr per length, plus a 10-bit lookahead table
  int32_t maxcode[18];
  int32_t valptr[17];
  int32_t mincode[17];
  uint8_t vals[256];
  uint16_t look[1 << 10];   // (length << 8) | value for codes <= 10 bits, 0 = not in table
  // fast AC: code + magnitude bits within 10 bits -> fac = (total_len << 8) | (run + 1), fac_val = value
  int16_t fac_val[1 << 10];
  uint16_t fac[1 << 10];
  bool present = false;
};

struct Info {
  int w = 0, h = 0, ncomp = 0;
  int hs[3] = {1, 1, 1}, vs[3] = {1, 1, 1}, tq[3] = {0, 0, 0}, id[3] = {0, 0, 0};
  int hmax = 1, vmax = 1, mcux = 0, mcuy = 0;
  int bw[3] = {0, 0, 0}, bh[3] = {0, 0, 0};   // padded block grid per component
  int restart = 0;
};

static bool build_huff(Huff& t, const uint8_t* counts, const uint8_t* vals, int nvals) {
  memset(t.look, 0, sizeof(t.look));
  memcpy(t.vals, vals, nvals);
  int code = 0, k = 0;
  for (int len = 1; len <= 16; ++len) {
    t.valptr[len] = k;
    t.mincode[len] = code;
    // reject an over-subscribed code space BEFORE any lookup entry of this length is written:
    // (code << shift) | f must stay inside the 1024-entry table, and every symbol must exist
    if (code + counts[len - 1] > (1 << len) || k + counts[len - 1] > nvals) return false;
    for (int i = 0; i < counts[len - 1]; ++i) {
      if (len <= 10) {
        const int shift = 10 - len;
        for (int f = 0; f < (1 << shift); ++f) t.look[(code << shift) | f] = (uint16_t)((len << 8) | vals[k]);
      }
      ++code;
      ++k;
    }
    t.maxcode[len] = counts[len - 1] ? code - 1 : -1;
    if (code > (1 << len)) return false;
    code <<= 1;
  }
  t.maxcode[17] = 0x7fffffff;
  // fast AC entries: run/size symbol + its magnitude bits all inside the 10-bit window
  memset(t.fac, 0, sizeof(t.fac));
  for (int i = 0; i < (1 << 10); ++i) {
    const uint16_t e = t.look[i];
    if (!e) continue;
    const int len = e >> 8, rs = e & 0xFF, run = rs >> 4, sz = rs & 15;
    if (sz == 0 || len + sz > 10) continue;
    const int m = (i >> (10 - len - sz)) & ((1 << sz) - 1);
    const int v = m < (1 << (sz - 1)) ? m - (1 << sz) + 1 : m;
    t.fac[i] = (uint16_t)(((len + sz) << 8) | (run + 1));
    t.fac_val[i] = (int16_t)v;
  }
  t.present = true;
  return k == nvals;
}

// Built tables keyed by their DHT bytes (class, counts, values). Encoders reuse a handful of
// tables (the Annex K defaults, or one optimised set per image source), so a per-thread cache
// turns the ~10 us rebuild of each 1024-entry lookup table per image into a memcmp.
struct HuffCache {
  struct Entry {
    uint8_t key[1 + 16 + 256];
    int klen;
    Huff h;
  };
  std::vector<std::unique_ptr<Entry>> e;
  size_t next = 0;

  const Huff* get(int tc, const uint8_t* counts, const uint8_t* vals, int nv) {
    const int klen = 1 + 16 + nv;
    for (auto& x : e)
      if (x->klen == klen && x->key[0] == (uint8_t)tc && !memcmp(x->key + 1, counts, 16) &&
          !memcmp(x->key + 17, vals, nv))
        return &x->h;
    std::unique_ptr<Entry> n(new Entry());
    n->klen = klen;
    n->key[0] = (uint8_t)tc;
    memcpy(n->key + 1, counts, 16);
    memcpy(n->key + 17, vals, nv);
    if (!build_huff(n->h, counts, vals, nv)) return nullptr;
    if (e.size() < 32) {
      e.push_back(std::move(n));
      return &e.back()->h;
    }
    e[next] = std::move(n);            // round-robin replacement
    const Huff* r = &e[next]->h;
    next = (next + 1) % e.size();
    return r;
  }
};

static HuffCache& huff_cache() {
  thread_local HuffCache c;
  return c;
}

struct Bits {
  const uint8_t* p;
  const uint8_t* end;
  uint64_t acc = 0;
  int n = 0;
  bool marker = false;   // hit a marker: feed zeros from here on

  void fill() {
    // fast path: 6 bytes with no 0xFF (no stuffing / marker) go in at once
    if (!marker && end - p >= 8 && n <= 16) {
      uint64_t w;
      memcpy(&w, p, 8);
      const uint64_t x = ~w;   // 0xFF bytes become 0x00
      if (((x - 0x0101010101010101ULL) & ~x & 0x8080808080808080ULL & 0x0000FFFFFFFFFFFFULL) == 0) {
        const uint64_t be = __builtin_bswap64(w) >> 16;   // first 6 bytes, big-endian
        acc |= be << (16 - n);
        n += 48;
        p += 6;
        return;
      }
    }
    while (n <= 56) {
      uint32_t b = 0;
      if (!marker && p < end) {
        b = *p;
        if (b == 0xFF) {
          const uint8_t nx = p + 1 < end ? p[1] : 0;
          if (nx == 0x00) {
            p += 2;
          } else {
            marker = true;   // restart or end-of-scan marker: leave it for the caller
            b = 0;
          }
        } else {
          ++p;
        }
      }
      acc |= (uint64_t)b << (56 - n);
      n += 8;
    }
  }
  int peek(int k) {
    if (n < k) fill();
    return (int)(acc >> (64 - k));
  }
  void skip(int k) {
    acc <<= k;
    n -= k;
  }
  int get(int k) {
    if (k == 0) return 0;
    const int v = peek(k);
    skip(k);
    return v;
  }
  void reset_at(const uint8_t* q) {
    p = q;
    acc = 0;
    n = 0;
    marker = false;
  }
};

static inline int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

static inline int decode_huff(Bits& b, const Huff& t) {
  const int look = b.peek(10);
  const uint16_t e = t.look[look];
  if (e) {
    b.skip(e >> 8);
    return e & 0xFF;
  }
  int code = b.peek(16);
  for (int len = 11; len <= 16; ++len) {
    const int c = code >> (16 - len);
    if (c <= t.maxcode[len]) {
      b.skip(len);
      return t.vals[t.valptr[len] + c - t.mincode[len]];
    }
  }
  return -1;
}

// one block: DC diff + AC run-lengths -> natural-order quantised coefficients written straight
// into the (zero-initialised) destination; short AC codes decode in one table lookup
static inline bool decode_block(Bits& b, const Huff& dc, const Huff& ac, int& pred, int16_t* out) {
  const int s = decode_huff(b, dc);
  if (s < 0 || s > 11) return false;
  pred += s ? extend(b.get(s), s) : 0;
  out[0] = (int16_t)pred;
  for (int k = 1; k < 64;) {
    const int look = b.peek(10);
    const uint16_t f = ac.fac[look];
    if (f) {
      b.skip(f >> 8);
      k += (f & 0xFF) - 1;
      if (k > 63) return false;
      out[kZigzag[k]] = ac.fac_val[look];
      ++k;
      continue;
    }
    const int rs = decode_huff(b, ac);
    if (rs < 0) return false;
    const int r = rs >> 4, sz = rs & 15;
    if (sz == 0) {
      if (r != 15) break;   // EOB
      k += 16;
      continue;
    }
    k += r;
    if (k > 63) return false;
    out[kZigzag[k]] = (int16_t)extend(b.get(sz), sz);
    ++k;
  }
  return true;
}

struct Decoder {
  Info info;
  uint16_t qt[4][64];
  bool qpresent[4] = {false, false, false, false};
  const Huff* dct[4] = {nullptr, nullptr, nullptr, nullptr};   // thread-local cache entries
  const Huff* act[4] = {nullptr, nullptr, nullptr, nullptr};
  std::vector<int16_t> coef[3];   // per component [bh][bw][64] (when no external destination)
  int16_t* dst[3] = {nullptr, nullptr, nullptr};   // external zeroed destination per component

  int16_t* plane(int c) { return dst[c] ? dst[c] : coef[c].data(); }

  // header_only: stop at the first SOS (geometry / tables known, nothing decoded)
  int run(const uint8_t* d, size_t n, bool header_only = false) {
    const uint8_t* p = d;
    const uint8_t* end = d + n;
    if (n < 4 || p[0] != 0xFF || p[1] != 0xD8) return E_MARKER;
    p += 2;
    bool frame = false;
    while (p < end) {
      while (p < end && *p != 0xFF) ++p;   // tolerate fill / garbage between segments
      while (p < end && *p == 0xFF) ++p;
      if (p >= end) return E_TRUNC;
      const uint8_t m = *p++;
      if (m == 0xD9) return frame ? OK : E_MARKER;                    // EOI
      if (m >= 0xD0 && m <= 0xD7) continue;                            // stray RST
      if (end - p < 2) return E_TRUNC;
      const int len = (p[0] << 8) | p[1];
      if (len < 2 || p + len > end) return E_TRUNC;
      const uint8_t* seg = p + 2;
      const int sl = len - 2;
      switch (m) {
        case 0xC0: case 0xC1: {
          // one frame per image: a second SOF (after a scan) would change the block grid the
          // destination planes were sized for -- reject it before any scan writes
          if (frame) return E_MARKER;
          if (sl < 6 || seg[0] != 8) return E_UNSUPPORTED;
          info.h = (seg[1] << 8) | seg[2];
          info.w = (seg[3] << 8) | seg[4];
          info.ncomp = seg[5];
          if (info.w <= 0 || info.h <= 0 || (info.ncomp != 1 && info.ncomp != 3) || sl < 6 + 3 * info.ncomp)
            return E_UNSUPPORTED;
          info.hmax = info.vmax = 1;
          for (int c = 0; c < info.ncomp; ++c) {
            info.id[c] = seg[6 + 3 * c];
            info.hs[c] = seg[7 + 3 * c] >> 4;
            info.vs[c] = seg[7 + 3 * c] & 15;
            info.tq[c] = seg[8 + 3 * c] & 3;
            if (info.hs[c] < 1 || info.hs[c] > 2 || info.vs[c] < 1 || info.vs[c] > 2) return E_UNSUPPORTED;
            info.hmax = std::max(info.hmax, info.hs[c]);
            info.vmax = std::max(info.vmax, info.vs[c]);
          }
          if (info.ncomp == 1) info.hs[0] = info.vs[0] = info.hmax = info.vmax = 1;
          info.mcux = (info.w + 8 * info.hmax - 1) / (8 * info.hmax);
          info.mcuy = (info.h + 8 * info.vmax - 1) / (8 * info.vmax);
          for (int c = 0; c < info.ncomp; ++c) {
            info.bw[c] = info.mcux * info.hs[c];
            info.bh[c] = info.mcuy * info.vs[c];
            if (!dst[c] && !header_only) coef[c].assign((size_t)info.bw[c] * info.bh[c] * 64, 0);
          }
          frame = true;
          break;
        }
        case 0xC2: case 0xC3: case 0xC5: case 0xC6: case 0xC7: case 0xC9: case 0xCA: case 0xCB: case 0xCD:
        case 0xCE: case 0xCF:
          return E_UNSUPPORTED;   // progressive / lossless / arithmetic
        case 0xDB: {   // DQT
          int o = 0;
          while (o < sl) {
            const int pq = seg[o] >> 4, tq = seg[o] & 3;
            ++o;
            if (pq > 1 || o + 64 * (pq + 1) > sl) return E_TABLE;
            for (int k = 0; k < 64; ++k) {
              const int v = pq ? (seg[o + 2 * k] << 8) | seg[o + 2 * k + 1] : seg[o + k];
              qt[tq][kZigzag[k]] = (uint16_t)v;
            }
            o += 64 * (pq + 1);
            qpresent[tq] = true;
          }
          break;
        }
        case 0xC4: {   // DHT
          int o = 0;
          while (o < sl) {
            if (o + 17 > sl) return E_TABLE;
            const int tc = seg[o] >> 4, th = seg[o] & 3;
            const uint8_t* counts = seg + o + 1;
            int nv = 0;
            for (int i = 0; i < 16; ++i) nv += counts[i];
            if (nv > 256 || o + 17 + nv > sl) return E_TABLE;
            if (!header_only) {   // geometry probes need no tables
              const Huff* h = huff_cache().get(tc ? 1 : 0, counts, seg + o + 17, nv);
              if (!h) return E_TABLE;
              (tc ? act[th] : dct[th]) = h;
            }
            o += 17 + nv;
          }
          break;
        }
        case 0xDD:
          if (sl < 2) return E_TABLE;
          info.restart = (seg[0] << 8) | seg[1];
          break;
        case 0xDA: {   // SOS + entropy-coded data
          if (!frame) return E_MARKER;
          if (header_only) return OK;
          if (sl < 1) return E_TRUNC;
          const int ns = seg[0];
          if (ns < 1 || ns > info.ncomp || sl < 1 + 2 * ns + 3) return E_UNSUPPORTED;
          int comps[3], td[3], ta[3];
          for (int i = 0; i < ns; ++i) {
            const int cid = seg[1 + 2 * i];
            comps[i] = -1;
            for (int c = 0; c < info.ncomp; ++c)
              if (info.id[c] == cid) comps[i] = c;
            if (comps[i] < 0) return E_MARKER;
            td[i] = seg[2 + 2 * i] >> 4;
            ta[i] = seg[2 + 2 * i] & 3;
            if (td[i] > 3 || !dct[td[i]] || !act[ta[i]]) return E_TABLE;
          }
          const uint8_t* q = p + len;
          const int rc = scan(q, end, ns, comps, td, ta, &q);
          if (rc != OK) return rc;
          p = q;
          continue;
        }
        default:
          break;   // APPn, COM, ...
      }
      p += len;
    }
    return frame ? OK : E_TRUNC;
  }

  int scan(const uint8_t* q, const uint8_t* end, int ns, const int* comps, const int* td, const int* ta,
           const uint8_t** out_end) {
    Bits b{q, end};
    int pred[3] = {0, 0, 0};
    int todo = info.restart;
    auto restart = [&]() -> bool {
      // byte-align and consume the RSTn marker the bit reader stopped at
      const uint8_t* r = b.p;
      while (r + 1 < end && !(r[0] == 0xFF && r[1] >= 0xD0 && r[1] <= 0xD7)) ++r;
      if (r + 1 >= end) return false;
      b.reset_at(r + 2);
      pred[0] = pred[1] = pred[2] = 0;
      todo = info.restart;
      return true;
    };
    if (ns == 1) {   // non-interleaved: the component's own block raster (unpadded)
      const int c = comps[0];
      const int cw = (info.w * info.hs[c] + info.hmax - 1) / info.hmax;
      const int chh = (info.h * info.vs[c] + info.vmax - 1) / info.vmax;
      const int nbx = (cw + 7) / 8, nby = (chh + 7) / 8;
      for (int by = 0; by < nby; ++by)
        for (int bx = 0; bx < nbx; ++bx) {
          if (info.restart && todo == 0 && !restart()) return E_TRUNC;
          if (!decode_block(b, *dct[td[0]], *act[ta[0]], pred[0], plane(c) + ((size_t)by * info.bw[c] + bx) * 64))
            return E_HUFF;
          --todo;
        }
    } else {
      for (int my = 0; my < info.mcuy; ++my)
        for (int mx = 0; mx < info.mcux; ++mx) {
          if (info.restart && todo == 0 && !restart()) return E_TRUNC;
          for (int i = 0; i < ns; ++i) {
            const int c = comps[i];
            for (int v = 0; v < info.vs[c]; ++v)
              for (int h = 0; h < info.hs[c]; ++h) {
                const size_t by = (size_t)my * info.vs[c] + v, bx = (size_t)mx * info.hs[c] + h;
                if (!decode_block(b, *dct[td[i]], *act[ta[i]], pred[i], plane(c) + (by * info.bw[c] + bx) * 64))
                  return E_HUFF;
              }
          }
          --todo;
        }
    }
    // continue after the scan: find the next marker that is not a stuffed byte / RST
    const uint8_t* r = b.p;
    while (r + 1 < end && !(r[0] == 0xFF && r[1] != 0x00 && !(r[1] >= 0xD0 && r[1] <= 0xD7))) ++r;
    *out_end = r;
    return OK;
  }
};

// Persistent decode threads: a batch used to spawn and join its own threads, ~30 us each, which
// at 16 threads is ~0.5 ms of every serving micro-batch on the reader thread. The pool keeps the
// threads parked on a condition variable; run(n, fn) wakes n-1 of them and the caller is the n-th.
class WorkPool {
 public:
  static WorkPool& get() {
    static WorkPool p;
    return p;
  }
  void run(int n, const std::function<void()>& fn) {
    std::lock_guard<std::mutex> one(run_mu_);   // one batch at a time
    const int helpers = std::max(0, n - 1);
    {
      std::lock_guard<std::mutex> g(mu_);
      while ((int)th_.size() < helpers) {
        const int idx = (int)th_.size();
        th_.emplace_back([this, idx] { loop(idx); });
      }
      fn_ = &fn;
      want_ = helpers;
      pending_ = helpers;
      ++gen_;
    }
    cv_.notify_all();
    fn();
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [&] { return pending_ == 0; });
    fn_ = nullptr;
  }
  ~WorkPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }

 private:
  void loop(int idx) {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> g(mu_);
    for (;;) {
      cv_.wait(g, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      if (idx >= want_) continue;
      const std::function<void()>* f = fn_;
      g.unlock();
      (*f)();
      g.lock();
      if (--pending_ == 0) done_cv_.notify_all();
    }
  }
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> th_;
  const std::function<void()>* fn_ = nullptr;
  int want_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// geometry key a batch must share: w, h, ncomp, sampling of each component
static std::vector<int> geom_key(const Info& i) {
  std::vector<int> k = {i.w, i.h, i.ncomp};
  for (int c = 0; c < i.ncomp; ++c) {
    k.push_back(i.hs[c]);
    k.push_back(i.vs[c]);
  }
  return k;
}

}  // namespace zoo_jpeg

#ifndef ZOO_RT_NO_PYTHON
// Batch entropy decode. Returns None when any image is unsupported or the geometries differ;
// otherwise a dict: w, h, ncomp, hs, vs, bw, bh (per component), coef int16 [N, total_blocks, 64]
// (component planes back to back, each [bh][bw] blocks), qt uint16 [N, ncomp, 64] (natural
// order), offsets (block offset of each component plane).
static py::object jpeg_batch_coeffs(const std::vector<py::bytes>& payloads, int nthreads, py::object out) {
  using namespace zoo_jpeg;
  const size_t N = payloads.size();
  if (N == 0) return py::none();
  std::vector<std::pair<const uint8_t*, size_t>> src(N);
  for (size_t i = 0; i < N; ++i) {
    char* ptr = nullptr;
    Py_ssize_t len = 0;
    if (PyBytes_AsStringAndSize(payloads[i].ptr(), &ptr, &len) != 0) throw py::error_already_set();
    src[i] = {reinterpret_cast<const uint8_t*>(ptr), (size_t)len};
  }
  // phase 1: headers (geometry, tables) of every image, single pass
  std::vector<Decoder> dec(N);
  for (size_t i = 0; i < N; ++i)
    if (dec[i].run(src[i].first, src[i].second, true) != OK) return py::none();
  const Info& f = dec[0].info;
  const auto key = geom_key(f);
  for (size_t i = 1; i < N; ++i)
    if (geom_key(dec[i].info) != key) return py::none();
  std::vector<int> offs(f.ncomp);
  size_t total = 0;
  for (int c = 0; c < f.ncomp; ++c) {
    offs[c] = (int)total;
    total += (size_t)f.bw[c] * f.bh[c];
  }
  // phase 2: entropy-decode straight into the zeroed output (the caller's buffer -- e.g. a pinned
  // host ring slot -- when given and large enough), images spread over the threads
  py::array_t<int16_t> coef;
  if (!out.is_none()) {
    auto o = py::array_t<int16_t, py::array::c_style>::ensure(out);
    if (!o || (size_t)o.size() < N * total * 64 || !o.writeable()) return py::none();
    coef = o;
  } else {
    coef = py::array_t<int16_t>({(py::ssize_t)N, (py::ssize_t)total, (py::ssize_t)64});
  }
  py::array_t<uint16_t> qt({(py::ssize_t)N, (py::ssize_t)f.ncomp, (py::ssize_t)64});
  int16_t* cp = coef.mutable_data();
  uint16_t* qp = qt.mutable_data();
  std::vector<int> rc(N, 0);
  {
    py::gil_scoped_release nogil;
    std::atomic<size_t> next{0};
    const int nt = std::max(1, std::min<int>(nthreads, (int)N));
    const std::function<void()> body = [&]() {
        for (size_t i = next++; i < N; i = next++) {
          int16_t* base = cp + (size_t)i * total * 64;
          memset(base, 0, total * 64 * sizeof(int16_t));
          Decoder d;
          for (int c = 0; c < f.ncomp; ++c) d.dst[c] = base + (size_t)offs[c] * 64;
          rc[i] = d.run(src[i].first, src[i].second);
          if (rc[i] == OK && geom_key(d.info) != key) rc[i] = E_GEOM;
          for (int c = 0; c < f.ncomp && rc[i] == OK; ++c) {
            if (!d.qpresent[d.info.tq[c]]) rc[i] = E_TABLE;
            else memcpy(qp + ((size_t)i * f.ncomp + c) * 64, d.qt[d.info.tq[c]], 64 * 2);
          }
        }
      };
    WorkPool::get().run(nt, body);
  }
  for (size_t i = 0; i < N; ++i)
    if (rc[i] != OK) return py::none();
  py::dict d;
  d["w"] = f.w;
  d["h"] = f.h;
  d["ncomp"] = f.ncomp;
  d["hs"] = std::vector<int>(f.hs, f.hs + f.ncomp);
  d["vs"] = std::vector<int>(f.vs, f.vs + f.ncomp);
  d["bw"] = std::vector<int>(f.bw, f.bw + f.ncomp);
  d["bh"] = std::vector<int>(f.bh, f.bh + f.ncomp);
  d["offsets"] = offs;
  d["hmax"] = f.hmax;
  d["vmax"] = f.vmax;
  d["coef"] = coef;
  d["qt"] = qt;
  return d;
}

// single-image status (0 = decodable on the GPU path) for diagnostics / tests
static int jpeg_probe(const py::bytes& payload) {
  std::string s(payload);
  zoo_jpeg::Decoder d;
  return d.run(reinterpret_cast<const uint8_t*>(s.data()), s.size());
}

void register_jpeg(py::module& m) {
  m.def("jpeg_batch_coeffs", &jpeg_batch_coeffs, py::arg("payloads"), py::arg("nthreads") = 8,
        py::arg("out") = py::none());
  m.def("jpeg_probe", &jpeg_probe);
}
#endif
