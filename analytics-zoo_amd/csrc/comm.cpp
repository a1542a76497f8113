// zoo C++ communication layer: RCCL communicators driven directly (not through
// torch.distributed's ProcessGroup), on whatever HIP stream is current -- GradSync's dedicated comm
// stream during the overlapped backward.
//
// Why a layer of our own: the gradient buckets of GradSync go out as the bf16
// wire's all-to-all + chunk sum + all-gather, or ZeRO-1's reduce-scatter / all-gather, one set of
// collectives per bucket as soon as the bucket is final. Through the ProcessGroup every call pays
// its Python/C++ dispatch, work-object creation and stream-event bookkeeping; here a bucket's
// collectives are plain RCCL calls enqueued on the caller's stream (ncclGroupStart/End around
// the per-bucket pair), with the channel count for the fully connected 7-link xGMI mesh set
// through the communicator config (ZooConfig.rccl_channels) instead of process-wide variables.
//
// The library is torch's own librccl (the same symbols libtorch_hip resolves), so one process
// never loads two RCCL builds. Bootstrap: rank 0 creates the unique id, the caller distributes
// it (zoo/parallel/comm.py: torch.distributed object broadcast over the existing group).
//
// Reference parity: BigDL AllReduceParameter's block-manager shuffle
// re-designed as RCCL collectives over xGMI.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <string>
#include <vector>

namespace {

struct ZComm {
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1;
};

std::mutex g_mu;
std::vector<ZComm*> g_comms;

void check_nccl(ncclResult_t r, const char* what) {
  TORCH_CHECK(r == ncclSuccess, what, ": ", ncclGetErrorString(r));
}

ZComm* get(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(h >= 0 && h < (int64_t)g_comms.size() && g_comms[h] != nullptr, "zoo comm: bad handle ", h);
  return g_comms[h];
}

ncclDataType_t dtype_of(const torch::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    default: TORCH_CHECK(false, "zoo comm: unsupported dtype ", t.scalar_type());
  }
  return ncclFloat32;
}

ncclRedOp_t op_of(const std::string& op) {
  if (op == "sum") return ncclSum;
  if (op == "avg") return ncclAvg;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  if (op == "prod") return ncclProd;
  TORCH_CHECK(false, "zoo comm: unknown reduction ", op);
  return ncclSum;
}

void req_dev(const torch::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "zoo comm: ", what, " must be a contiguous GPU tensor");
}

hipStream_t cur() { return c10::hip::getCurrentHIPStream().stream(); }

// A one-rank communicator's collectives are identities: a device copy on the current stream (or
// nothing, in place) instead of an RCCL launch. Keeps world-1 runs (force_comm, tests) free of
// RCCL's single-rank paths, which a hipGraph capture of an all-to-all left hanging at communicator
// teardown (profiles/r6/rccl_capture_probe_all_to_all_r6.log).
bool local_copy(const ZComm* c, void* dst, const void* src, size_t bytes) {
  if (c->world != 1) return false;
  if (dst != src && bytes > 0)
    TORCH_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, cur()) == hipSuccess,
                "zoo comm: local copy failed");
  return true;
}

}  // namespace

py::bytes comm_unique_id() {
  ncclUniqueId id;
  check_nccl(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return py::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
}

// channels > 0: minimum (and maximum) RCCL channels of this communicator
int64_t comm_init(py::bytes uid, int64_t world, int64_t rank, int64_t channels) {
  std::string s = uid;
  TORCH_CHECK(s.size() == sizeof(ncclUniqueId), "comm_init: unique id must be ", sizeof(ncclUniqueId), " bytes");
  TORCH_CHECK(world >= 1 && rank >= 0 && rank < world, "comm_init: rank / world");
  ncclUniqueId id;
  std::memcpy(&id, s.data(), sizeof(id));
  auto* c = new ZComm();
  c->rank = (int)rank;
  c->world = (int)world;
  ncclResult_t r;
  if (channels > 0) {
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.minCTAs = (int)channels;
    cfg.maxCTAs = (int)channels;
    r = ncclCommInitRankConfig(&c->comm, (int)world, id, (int)rank, &cfg);
  } else {
    r = ncclCommInitRank(&c->comm, (int)world, id, (int)rank);
  }
  if (r != ncclSuccess) {
    delete c;
    check_nccl(r, "ncclCommInitRankConfig");
  }
  std::lock_guard<std::mutex> lk(g_mu);
  g_comms.push_back(c);
  return (int64_t)g_comms.size() - 1;
}

void comm_destroy(int64_t h) {
  ZComm* c = get(h);
  {
    std::lock_guard<std::mutex> lk(g_mu);
    g_comms[h] = nullptr;
  }
  if (c->comm) ncclCommDestroy(c->comm);
  delete c;
}

std::vector<int64_t> comm_info(int64_t h) {
  ZComm* c = get(h);
  return {c->rank, c->world};
}

void comm_all_reduce(int64_t h, torch::Tensor t, const std::string& op) {
  ZComm* c = get(h);
  req_dev(t, "all_reduce tensor");
  if (local_copy(c, t.data_ptr(), t.data_ptr(), 0)) return;
  check_nccl(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), dtype_of(t), op_of(op), c->comm, cur()),
             "ncclAllReduce");
}

// out [n / world] = this rank's chunk of the sum of every rank's inp [n]
void comm_reduce_scatter(int64_t h, torch::Tensor out, torch::Tensor inp, const std::string& op) {
  ZComm* c = get(h);
  req_dev(out, "reduce_scatter out");
  req_dev(inp, "reduce_scatter input");
  TORCH_CHECK(out.scalar_type() == inp.scalar_type() && inp.numel() == out.numel() * c->world,
              "reduce_scatter: input must hold world x out elements of the same dtype");
  if (local_copy(c, out.data_ptr(), inp.data_ptr(), out.nbytes())) return;
  check_nccl(ncclReduceScatter(inp.data_ptr(), out.data_ptr(), out.numel(), dtype_of(out), op_of(op), c->comm, cur()),
             "ncclReduceScatter");
}

// out [world * n] = every rank's inp [n], in rank order
void comm_all_gather(int64_t h, torch::Tensor out, torch::Tensor inp) {
  ZComm* c = get(h);
  req_dev(out, "all_gather out");
  req_dev(inp, "all_gather input");
  TORCH_CHECK(out.scalar_type() == inp.scalar_type() && out.numel() == inp.numel() * c->world,
              "all_gather: out must hold world x input elements of the same dtype");
  if (local_copy(c, out.data_ptr(), inp.data_ptr(), out.nbytes())) return;
  check_nccl(ncclAllGather(inp.data_ptr(), out.data_ptr(), inp.numel(), dtype_of(inp), c->comm, cur()),
             "ncclAllGather");
}

// chunk j of inp [world * n] goes to rank j; chunk i of out is what rank i sent here
void comm_all_to_all(int64_t h, torch::Tensor out, torch::Tensor inp) {
  ZComm* c = get(h);
  req_dev(out, "all_to_all out");
  req_dev(inp, "all_to_all input");
  TORCH_CHECK(out.scalar_type() == inp.scalar_type() && out.numel() == inp.numel() && inp.numel() % c->world == 0,
              "all_to_all: equal-size tensors of the same dtype, divisible by the world size");
  if (local_copy(c, out.data_ptr(), inp.data_ptr(), out.nbytes())) return;
  check_nccl(ncclAllToAll(inp.data_ptr(), out.data_ptr(), inp.numel() / c->world, dtype_of(inp), c->comm, cur()),
             "ncclAllToAll");
}

void comm_broadcast(int64_t h, torch::Tensor t, int64_t root) {
  ZComm* c = get(h);
  req_dev(t, "broadcast tensor");
  TORCH_CHECK(root >= 0 && root < c->world, "broadcast: root");
  if (local_copy(c, t.data_ptr(), t.data_ptr(), 0)) return;
  check_nccl(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), dtype_of(t), (int)root, c->comm, cur()),
             "ncclBroadcast");
}

// fuse the collectives issued between the two calls into one RCCL launch group
void comm_group_start() { check_nccl(ncclGroupStart(), "ncclGroupStart"); }
void comm_group_end() { check_nccl(ncclGroupEnd(), "ncclGroupEnd"); }

void register_comm(py::module& m) {
  m.def("comm_unique_id", &comm_unique_id);
  m.def("comm_init", &comm_init, py::arg("uid"), py::arg("world"), py::arg("rank"), py::arg("channels") = 0);
  m.def("comm_destroy", &comm_destroy);
  m.def("comm_info", &comm_info);
  m.def("comm_all_reduce", &comm_all_reduce, py::arg("h"), py::arg("t"), py::arg("op") = "sum");
  m.def("comm_reduce_scatter", &comm_reduce_scatter, py::arg("h"), py::arg("out"), py::arg("inp"),
        py::arg("op") = "sum");
  m.def("comm_all_gather", &comm_all_gather);
  m.def("comm_all_to_all", &comm_all_to_all);
  m.def("comm_broadcast", &comm_broadcast);
  m.def("comm_group_start", &comm_group_start);
  m.def("comm_group_end", &comm_group_end);
}
