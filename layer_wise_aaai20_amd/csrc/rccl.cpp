// Native RCCL communicator for the gradient-bucket collectives (torch.ops.lwaaai.rccl_*).
//
// The bucket exchange of the reference is one blocking NCCL call per tensor from Python
// (CIFAR10/core.py:218, IMAGENET/training/train_imagenet_nv.py:298,385). Here the engine issues
// one collective per bucket from its side HIP stream (parallel/engine.py) and, once warm, the
// whole training step — collectives included — is replayed as one HIP graph
// (train/graphs.py). Going through c10d for those calls puts a Work object with HIP events on
// the ProcessGroup watchdog's list; on ROCm that thread can query an event last recorded inside
// the capture and abort the process (hipErrorCapturedEvent, profiles/r2_rccl_capture_race.log).
// These ops call RCCL directly on the caller's current stream: stream-ordered, no Work, no
// watchdog, capturable. The communicator is created from a unique id that rank 0 broadcasts
// over the existing process group; c10d keeps everything else (barriers, init-time checks).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>
#include <rccl/rccl.h>
#include <torch/library.h>

#include <cstring>

namespace {

using at::Tensor;

inline hipStream_t cur_stream() {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
}

void check(ncclResult_t r, const char* what) {
  TORCH_CHECK(r == ncclSuccess, "RCCL ", what, " failed: ", ncclGetErrorString(r));
}

ncclDataType_t dtype_of(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    case at::kHalf: return ncclFloat16;
    case at::kBFloat16: return ncclBfloat16;
    case at::kDouble: return ncclFloat64;
    default: TORCH_CHECK(false, "rccl: unsupported dtype ", t.scalar_type());
  }
}

ncclComm_t comm_of(int64_t h) {
  TORCH_CHECK(h != 0, "rccl: communicator not initialised");
  return reinterpret_cast<ncclComm_t>(h);
}

void check_dev(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "rccl: ", name, " must be a contiguous GPU tensor");
}

Tensor rccl_unique_id() {
  ncclUniqueId id;
  check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  Tensor out = at::empty({NCCL_UNIQUE_ID_BYTES}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(out.data_ptr(), &id, NCCL_UNIQUE_ID_BYTES);
  return out;
}

int64_t rccl_init(Tensor uid, int64_t world, int64_t rank, int64_t device) {
  TORCH_CHECK(uid.device().is_cpu() && uid.scalar_type() == at::kByte &&
                  uid.numel() == NCCL_UNIQUE_ID_BYTES && uid.is_contiguous(),
              "rccl_init: uid must be a contiguous CPU uint8 tensor of ", NCCL_UNIQUE_ID_BYTES,
              " bytes");
  TORCH_CHECK(world >= 1 && rank >= 0 && rank < world, "rccl_init: bad rank/world");
  const c10::DeviceGuard guard(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  ncclUniqueId id;
  std::memcpy(&id, uid.data_ptr(), NCCL_UNIQUE_ID_BYTES);
  ncclComm_t comm = nullptr;
  check(ncclCommInitRank(&comm, (int)world, id, (int)rank), "ncclCommInitRank");
  return reinterpret_cast<int64_t>(comm);
}

void rccl_destroy(int64_t h) {
  if (h != 0) check(ncclCommDestroy(comm_of(h)), "ncclCommDestroy");
}

void rccl_all_gather(int64_t h, Tensor send, Tensor recv) {
  check_dev(send, "send");
  check_dev(recv, "recv");
  TORCH_CHECK(send.scalar_type() == recv.scalar_type(), "rccl_all_gather: dtype mismatch");
  int n = 0;
  check(ncclCommCount(comm_of(h), &n), "ncclCommCount");
  TORCH_CHECK(recv.numel() == send.numel() * n, "rccl_all_gather: recv must hold world * send");
  const c10::DeviceGuard guard(send.device());
  check(ncclAllGather(send.data_ptr(), recv.data_ptr(), (size_t)send.numel(), dtype_of(send),
                      comm_of(h), cur_stream()),
        "ncclAllGather");
}

void rccl_all_reduce(int64_t h, Tensor t, int64_t op) {
  check_dev(t, "tensor");
  const c10::DeviceGuard guard(t.device());
  const ncclRedOp_t rop = op == 1 ? ncclMax : (op == 2 ? ncclMin : ncclSum);
  check(ncclAllReduce(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), dtype_of(t), rop,
                      comm_of(h), cur_stream()),
        "ncclAllReduce");
}

void rccl_broadcast(int64_t h, Tensor t, int64_t root) {
  check_dev(t, "tensor");
  const c10::DeviceGuard guard(t.device());
  check(ncclBroadcast(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), dtype_of(t), (int)root,
                      comm_of(h), cur_stream()),
        "ncclBroadcast");
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(lwaaai, m) {
  m.def("rccl_unique_id() -> Tensor", &rccl_unique_id);
  m.def("rccl_init(Tensor uid, int world, int rank, int device) -> int", &rccl_init);
  m.def("rccl_destroy(int comm) -> ()", &rccl_destroy);
  m.def("rccl_all_gather(int comm, Tensor send, Tensor(a!) recv) -> ()", &rccl_all_gather);
  m.def("rccl_all_reduce(int comm, Tensor(a!) t, int op) -> ()", &rccl_all_reduce);
  m.def("rccl_broadcast(int comm, Tensor(a!) t, int root) -> ()", &rccl_broadcast);
}
