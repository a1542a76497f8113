// zoo host runtime (C++): the native pieces of the reference's data layer,
// observability and model IO that are not GPU kernels.
//
//  * Gatherer — a fixed worker pool that assembles minibatches by copying
//    rows of a contiguous host array in a (shuffled) index order into a
//    destination buffer (typically a pinned host tensor that is then copied to
//    HBM with a non-blocking DMA). Jobs are asynchronous (submit -> ticket ->
//    wait) so batch k+1 is gathered while the GPU runs batch k. This replaces
//    the reference's SampleToMiniBatch / MTSampleToMiniBatch
//    (Zs/feature/common/MTSampleToMiniBatch.scala:28-139) and the cached
//    FeatureSet iterator (Zs/feature/FeatureSet.scala:230-330).
//  * crc32c / masked_crc32c / tfrecord_frame — TFRecord framing for the
//    TensorBoard event writer (Zs/tensorboard/RecordWriter.scala:30-90).
//  * pb_fields — a protobuf wire-format scanner used by the BigDL ``.model``
//    codec (zoo/utils/bigdl_proto.py) to walk nested messages without protoc.
//  * NativeStore (serving.cpp) — the Cluster Serving queue: Redis-protocol
//    streams/hashes with a TCP front end and GIL-free worker fast paths.
//
// Everything above the Python bindings is plain C++17: with -DZOO_RT_NO_PYTHON the file
// compiles without pybind11 so tools/sanitize_runtime.py can build it into a standalone
// ASan/UBSan/TSan self-test (csrc/runtime/selftest/rt_selftest.cpp).
#ifndef ZOO_RT_NO_PYTHON
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
namespace py = pybind11;
#define ZOO_RT_NOGIL py::gil_scoped_release nogil_
#else
#define ZOO_RT_NOGIL (void)0
#endif

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

// ------------------------------------------------------------------ Gatherer
class Gatherer {
 public:
  explicit Gatherer(int nthreads) : stop_(false), next_ticket_(1) {
    if (nthreads < 1) nthreads = 1;
    for (int i = 0; i < nthreads; ++i) workers_.emplace_back([this] { loop(); });
  }
  ~Gatherer() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

  int num_threads() const { return (int)workers_.size(); }

  // Copy rows src[idx[i]] -> dst[i] for i in [0, n). Synchronous, parallel.
  void gather(uintptr_t src, int64_t nrows, int64_t row_bytes, uintptr_t idx, int64_t n, uintptr_t dst) {
    const int64_t t = submit(src, nrows, row_bytes, idx, n, dst);
    wait(t);
  }

  int64_t submit(uintptr_t src, int64_t nrows, int64_t row_bytes, uintptr_t idx, int64_t n, uintptr_t dst) {
    const int64_t* ip = reinterpret_cast<const int64_t*>(idx);
    for (int64_t i = 0; i < n; ++i)
      if (ip[i] < 0 || ip[i] >= nrows) throw std::out_of_range("Gatherer: index out of range");
    const int parts = std::max<int64_t>(1, std::min<int64_t>((int64_t)workers_.size(), n / 64 + 1));
    std::lock_guard<std::mutex> g(mu_);
    const int64_t ticket = next_ticket_++;
    pending_[ticket] = parts;
    const int64_t chunk = (n + parts - 1) / parts;
    for (int p = 0; p < parts; ++p) {
      const int64_t lo = p * chunk, hi = std::min(n, lo + chunk);
      jobs_.push_back([=] {
        const char* s = reinterpret_cast<const char*>(src);
        char* d = reinterpret_cast<char*>(dst);
        for (int64_t i = lo; i < hi; ++i) std::memcpy(d + i * row_bytes, s + ip[i] * row_bytes, row_bytes);
        finish(ticket);
      });
    }
    cv_.notify_all();
    return ticket;
  }

  void wait(int64_t ticket) {
    ZOO_RT_NOGIL;
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [&] { return pending_.find(ticket) == pending_.end(); });
  }

  bool ready(int64_t ticket) {
    std::lock_guard<std::mutex> g(mu_);
    return pending_.find(ticket) == pending_.end();
  }

 private:
  void finish(int64_t ticket) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = pending_.find(ticket);
    if (it != pending_.end() && --it->second == 0) {
      pending_.erase(it);
      done_cv_.notify_all();
    }
  }

  void loop() {
    for (;;) {
      std::function<void()> job;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || !jobs_.empty(); });
        if (stop_ && jobs_.empty()) return;
        job = std::move(jobs_.front());
        jobs_.pop_front();
      }
      job();
    }
  }

  std::vector<std::thread> workers_;
  std::deque<std::function<void()>> jobs_;
  std::unordered_map<int64_t, int> pending_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  bool stop_;
  int64_t next_ticket_;
};

// ------------------------------------------------------------------ CRC32C
uint32_t crc_table[8][256];
std::once_flag crc_once;

void init_crc() {
  const uint32_t poly = 0x82F63B78u;  // Castagnoli, reflected
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ poly : c >> 1;
    crc_table[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i)
    for (int t = 1; t < 8; ++t) crc_table[t][i] = (crc_table[t - 1][i] >> 8) ^ crc_table[0][crc_table[t - 1][i] & 0xff];
}

uint32_t crc32c_raw(const uint8_t* p, size_t n) {
  std::call_once(crc_once, init_crc);  // writer threads may race to the first CRC
  uint32_t c = 0xFFFFFFFFu;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    v ^= c;
    c = crc_table[7][v & 0xff] ^ crc_table[6][(v >> 8) & 0xff] ^ crc_table[5][(v >> 16) & 0xff] ^
        crc_table[4][(v >> 24) & 0xff] ^ crc_table[3][(v >> 32) & 0xff] ^ crc_table[2][(v >> 40) & 0xff] ^
        crc_table[1][(v >> 48) & 0xff] ^ crc_table[0][(v >> 56) & 0xff];
    p += 8;
    n -= 8;
  }
  while (n--) c = crc_table[0][(c ^ *p++) & 0xff] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

uint32_t mask_crc(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }

// TFRecord: uint64 length | uint32 masked_crc(length) | data | uint32 masked_crc(data)
std::string tfrecord_frame_raw(const std::string& s) {
  std::string out;
  out.resize(12 + s.size() + 4);
  uint64_t len = s.size();
  std::memcpy(&out[0], &len, 8);
  uint32_t lc = mask_crc(crc32c_raw(reinterpret_cast<const uint8_t*>(&len), 8));
  std::memcpy(&out[8], &lc, 4);
  std::memcpy(&out[12], s.data(), s.size());
  uint32_t dc = mask_crc(crc32c_raw(reinterpret_cast<const uint8_t*>(s.data()), s.size()));
  std::memcpy(&out[12 + s.size()], &dc, 4);
  return out;
}

// ------------------------------------------------------------------ protobuf
// One wire-format field: varint/fixed values in `v`, length-delimited payloads as
// [off, off + v) into the scanned buffer.
struct PbField {
  int field, wt;
  uint64_t v;
  size_t off;
};

void pb_scan(const uint8_t* base, size_t size, std::vector<PbField>* out) {
  const uint8_t* p = base;
  const uint8_t* end = base + size;
  auto varint = [&](uint64_t& v) {
    v = 0;
    int shift = 0;
    while (p < end) {
      uint8_t c = *p++;
      v |= (uint64_t)(c & 0x7f) << shift;
      if (!(c & 0x80)) return;
      shift += 7;
      if (shift > 63) throw std::runtime_error("pb: varint too long");
    }
    throw std::runtime_error("pb: truncated varint");
  };
  while (p < end) {
    uint64_t key;
    varint(key);
    PbField f{(int)(key >> 3), (int)(key & 7), 0, 0};
    if (f.wt == 0) {
      varint(f.v);
    } else if (f.wt == 1) {
      if (end - p < 8) throw std::runtime_error("pb: truncated fixed64");
      std::memcpy(&f.v, p, 8);
      p += 8;
    } else if (f.wt == 2) {
      varint(f.v);
      if ((uint64_t)(end - p) < f.v) throw std::runtime_error("pb: truncated bytes");
      f.off = (size_t)(p - base);
      p += f.v;
    } else if (f.wt == 5) {
      if (end - p < 4) throw std::runtime_error("pb: truncated fixed32");
      uint32_t v;
      std::memcpy(&v, p, 4);
      f.v = v;
      p += 4;
    } else {
      throw std::runtime_error("pb: unsupported wire type " + std::to_string(f.wt));
    }
    out->push_back(f);
  }
}

#ifndef ZOO_RT_NO_PYTHON
uint32_t crc32c(py::bytes b) {
  std::string s = b;
  return crc32c_raw(reinterpret_cast<const uint8_t*>(s.data()), s.size());
}

uint32_t masked_crc32c(py::bytes b) {
  std::string s = b;
  return mask_crc(crc32c_raw(reinterpret_cast<const uint8_t*>(s.data()), s.size()));
}

py::bytes tfrecord_frame(py::bytes b) { return py::bytes(tfrecord_frame_raw(std::string(b))); }

// Returns [(field_number, wire_type, value)] where value is an int for
// varint/fixed and bytes for length-delimited fields.
py::list pb_fields(py::bytes b) {
  std::string s = b;
  std::vector<PbField> fs;
  pb_scan(reinterpret_cast<const uint8_t*>(s.data()), s.size(), &fs);
  py::list out;
  for (const auto& f : fs) {
    if (f.wt == 2) out.append(py::make_tuple(f.field, f.wt, py::bytes(s.data() + f.off, (size_t)f.v)));
    else out.append(py::make_tuple(f.field, f.wt, py::int_(f.v)));
  }
  return out;
}
#endif

}  // namespace

#ifndef ZOO_RT_NO_PYTHON
void register_serving(py::module& m);  // serving.cpp
void register_jpeg(py::module& m);     // jpeg.cpp

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "zoo native host runtime (batch gather, TFRecord/CRC32C, protobuf wire scanner, serving queue)";
  register_serving(m);
  register_jpeg(m);
  py::class_<Gatherer>(m, "Gatherer")
      .def(py::init<int>(), py::arg("nthreads") = 4)
      .def("gather", &Gatherer::gather)
      .def("submit", &Gatherer::submit)
      .def("wait", &Gatherer::wait)
      .def("ready", &Gatherer::ready)
      .def_property_readonly("num_threads", &Gatherer::num_threads);
  m.def("crc32c", &crc32c);
  m.def("masked_crc32c", &masked_crc32c);
  m.def("tfrecord_frame", &tfrecord_frame);
  m.def("pb_fields", &pb_fields);
}
#endif  // ZOO_RT_NO_PYTHON
