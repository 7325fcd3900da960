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

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>
#include <unistd.h>

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

// An RCCL call on a non-blocking communicator may return ncclInProgress: poll the communicator
// state until the call has completed (or failed). Blocking communicators never return it.
ncclResult_t settle(ncclComm_t comm, ncclResult_t r) {
  while (r == ncclInProgress) {
    std::this_thread::yield();
    if (ncclCommGetAsyncError(comm, &r) != ncclSuccess) return ncclInternalError;
  }
  return r;
}

// timeout_s > 0: the blocking ncclCommInitRank runs on a helper thread and this call waits for
// it against a deadline. A peer that never joins (a rank that failed before reaching the init,
// after the ranks agreed to create the communicator) would otherwise block this rank inside the
// init forever; here the call raises instead (the helper thread is left behind, blocked, and its
// communicator — should the init ever complete — is never used), so the rank reaches the fallback
// agreement (parallel/comm.py _init_native_agreed). The communicator itself is an ordinary
// BLOCKING one (a non-blocking one, ncclConfig_t.blocking = 0, lets any call return
// ncclInProgress and finish its launch later, which a captured step should not depend on).
// timeout_s <= 0: the init on this thread, no deadline.
namespace {
struct InitJob {
  std::mutex mu;
  bool done = false;
  bool abandoned = false;
  ncclResult_t r = ncclSuccess;
  ncclComm_t comm = nullptr;
};
}  // namespace

int64_t rccl_init(Tensor uid, int64_t world, int64_t rank, int64_t device, double timeout_s) {
  TORCH_CHECK(uid.device().is_cpu() && uid.scalar_type() == at::kByte &&
                  uid.numel() == NCCL_UNIQUE_ID_BYTES && uid.is_contiguous(),
              "rccl_init: uid must be a contiguous CPU uint8 tensor of ", NCCL_UNIQUE_ID_BYTES,
              " bytes");
  TORCH_CHECK(world >= 1 && rank >= 0 && rank < world, "rccl_init: bad rank/world");
  const c10::DeviceGuard guard(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  ncclUniqueId id;
  std::memcpy(&id, uid.data_ptr(), NCCL_UNIQUE_ID_BYTES);
  if (timeout_s <= 0) {
    ncclComm_t comm = nullptr;
    check(ncclCommInitRank(&comm, (int)world, id, (int)rank), "ncclCommInitRank");
    return reinterpret_cast<int64_t>(comm);
  }
  auto job = std::make_shared<InitJob>();
  std::thread([job, id, world, rank, device]() {
    hipSetDevice((int)device);
    ncclComm_t comm = nullptr;
    const ncclResult_t r = ncclCommInitRank(&comm, (int)world, id, (int)rank);
    std::lock_guard<std::mutex> lk(job->mu);
    job->r = r;
    job->comm = comm;
    job->done = true;
  }).detach();
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    {
      std::lock_guard<std::mutex> lk(job->mu);
      if (job->done) {
        TORCH_CHECK(job->r == ncclSuccess, "RCCL ncclCommInitRank failed: ",
                    ncclGetErrorString(job->r));
        return reinterpret_cast<int64_t>(job->comm);
      }
      const double waited =
          std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (waited > timeout_s) {
        job->abandoned = true;
        TORCH_CHECK(false, "ncclCommInitRank: not complete after ", waited,
                    " s (a peer rank never joined); communicator abandoned");
      }
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
  }
}

void rccl_destroy(int64_t h) {
  if (h != 0) check(ncclCommDestroy(comm_of(h)), "ncclCommDestroy");
}

// Local, non-blocking teardown: ncclCommDestroy finalizes the communicator, which waits on the
// peers (it hung a 2-rank test whose ranks tore down in different orders around c10d's own
// destroy); ncclCommAbort frees it without any peer involvement.
void rccl_abort(int64_t h) {
  if (h != 0) check(ncclCommAbort(comm_of(h)), "ncclCommAbort");
}

void rccl_all_gather(int64_t h, Tensor send, Tensor recv) {
  check_dev(send, "send");
  check_dev(recv, "recv");
  TORCH_CHECK(send.scalar_type() == recv.scalar_type(), "rccl_all_gather: dtype mismatch");
  int n = 0;
  check(ncclCommCount(comm_of(h), &n), "ncclCommCount");
  TORCH_CHECK(recv.numel() == send.numel() * n, "rccl_all_gather: recv must hold world * send");
  const c10::DeviceGuard guard(send.device());
  check(settle(comm_of(h), ncclAllGather(send.data_ptr(), recv.data_ptr(), (size_t)send.numel(),
                                         dtype_of(send), comm_of(h), cur_stream())),
        "ncclAllGather");
}

void rccl_all_reduce(int64_t h, Tensor t, int64_t op) {
  check_dev(t, "tensor");
  const c10::DeviceGuard guard(t.device());
  const ncclRedOp_t rop = op == 1 ? ncclMax : (op == 2 ? ncclMin : ncclSum);
  check(settle(comm_of(h), ncclAllReduce(t.data_ptr(), t.data_ptr(), (size_t)t.numel(),
                                         dtype_of(t), rop, comm_of(h), cur_stream())),
        "ncclAllReduce");
}

void rccl_broadcast(int64_t h, Tensor t, int64_t root) {
  check_dev(t, "tensor");
  const c10::DeviceGuard guard(t.device());
  check(settle(comm_of(h), ncclBroadcast(t.data_ptr(), t.data_ptr(), (size_t)t.numel(),
                                         dtype_of(t), (int)root, comm_of(h), cur_stream())),
        "ncclBroadcast");
}

// Grouped point-to-point transfers: every send and receive of the two lists inside one
// ncclGroupStart / ncclGroupEnd, so RCCL schedules them together over the xGMI links (one
// channel set per peer) instead of serialising them; sends to and receives from this rank itself
// are allowed (a local copy). Pairs must match across ranks in count, size and dtype, in order
// per peer — what the all-to-all and variable-size all-gather of the quantised reduce-scatter
// wire (compress/codecs.py QuantRSCodec) are built from. Empty tensors are skipped on both sides.
void rccl_send_recv(int64_t h, std::vector<Tensor> sends, std::vector<int64_t> send_peers,
                    std::vector<Tensor> recvs, std::vector<int64_t> recv_peers) {
  TORCH_CHECK(sends.size() == send_peers.size() && recvs.size() == recv_peers.size(),
              "rccl_send_recv: one peer per tensor");
  int n = 0;
  check(ncclCommCount(comm_of(h), &n), "ncclCommCount");
  for (size_t i = 0; i < sends.size(); ++i) {
    check_dev(sends[i], "send");
    TORCH_CHECK(send_peers[i] >= 0 && send_peers[i] < n, "rccl_send_recv: bad send peer");
  }
  for (size_t i = 0; i < recvs.size(); ++i) {
    check_dev(recvs[i], "recv");
    TORCH_CHECK(recv_peers[i] >= 0 && recv_peers[i] < n, "rccl_send_recv: bad recv peer");
  }
  if (sends.empty() && recvs.empty()) return;
  const c10::DeviceGuard guard((sends.empty() ? recvs[0] : sends[0]).device());
  ncclComm_t c = comm_of(h);
  hipStream_t st = cur_stream();
  check(ncclGroupStart(), "ncclGroupStart");
  for (size_t i = 0; i < sends.size(); ++i)
    if (sends[i].numel() > 0)
      check(ncclSend(sends[i].data_ptr(), (size_t)sends[i].numel(), dtype_of(sends[i]),
                     (int)send_peers[i], c, st), "ncclSend");
  for (size_t i = 0; i < recvs.size(); ++i)
    if (recvs[i].numel() > 0)
      check(ncclRecv(recvs[i].data_ptr(), (size_t)recvs[i].numel(), dtype_of(recvs[i]),
                     (int)recv_peers[i], c, st), "ncclRecv");
  check(settle(c, ncclGroupEnd()), "ncclGroupEnd (send/recv)");
}

// Equal-chunk all-to-all: chunk q of `send` goes to rank q, chunk q of `recv` comes from rank q.
void rccl_all_to_all(int64_t h, Tensor send, Tensor recv) {
  check_dev(send, "send");
  check_dev(recv, "recv");
  int n = 0;
  check(ncclCommCount(comm_of(h), &n), "ncclCommCount");
  TORCH_CHECK(send.scalar_type() == recv.scalar_type() && send.numel() == recv.numel() &&
                  send.numel() % n == 0, "rccl_all_to_all: send / recv must be world equal chunks");
  const int64_t chunk = send.numel() / n;
  std::vector<Tensor> s, r;
  std::vector<int64_t> p;
  for (int q = 0; q < n; ++q) {
    s.push_back(send.narrow(0, q * chunk, chunk));
    r.push_back(recv.narrow(0, q * chunk, chunk));
    p.push_back(q);
  }
  rccl_send_recv(h, s, p, r, p);
}

// Reduce-scatter: recv (numel = send / world) gets this rank's chunk of the element-wise reduction.
void rccl_reduce_scatter(int64_t h, Tensor send, Tensor recv, int64_t op) {
  check_dev(send, "send");
  check_dev(recv, "recv");
  int n = 0;
  check(ncclCommCount(comm_of(h), &n), "ncclCommCount");
  TORCH_CHECK(send.scalar_type() == recv.scalar_type() && send.numel() == recv.numel() * n,
              "rccl_reduce_scatter: send must hold world * recv");
  const c10::DeviceGuard guard(send.device());
  const ncclRedOp_t rop = op == 1 ? ncclMax : (op == 2 ? ncclMin : ncclSum);
  check(settle(comm_of(h), ncclReduceScatter(send.data_ptr(), recv.data_ptr(), (size_t)recv.numel(),
                                             dtype_of(send), rop, comm_of(h), cur_stream())),
        "ncclReduceScatter");
}

// ---------------------------------------------------------------------------------------------
// Watchdog. c10d's ProcessGroup watchdog never sees these collectives (they bypass c10d), so a rank
// that stops participating — a crashed peer, a rank whose control flow diverged, a mismatched
// bucket plan at run time — would leave every other rank blocked inside an RCCL kernel forever,
// silently, inside a replayed graph. One host thread per communicator:
//   * polls ncclCommGetAsyncError (RCCL's own error reporting: peer loss, IB/xGMI errors);
//   * enforces a deadline on the last step "mark": an event recorded on the compute stream after
//     each step (outside any graph capture: an event recorded inside a capture must not be
//     queried). If it has not completed `timeout` seconds after it was recorded, the step is
//     declared hung.
// On failure: action 0 (training) prints the reason, aborts the communicator (which makes the
// blocked RCCL kernels return) and ends the process with exit code 86 — the launcher sees a
// non-zero exit instead of a hang; action 1 (tests) only records the failure for check().
// Reference failure handling: train_imagenet_nv.py:161-163 (world-size assert), :704-716 (top-level
// catch and log).
struct Watchdog {
  ncclComm_t comm = nullptr;
  int device = 0;
  double timeout_s = 600.0;
  int action = 0;
  std::mutex mu;
  hipEvent_t ev = nullptr;
  bool pending = false;
  std::chrono::steady_clock::time_point t_mark;
  std::atomic<int> fired{0};
  std::atomic<bool> stop{false};
  std::string why;
  std::thread th;

  void fail(const std::string& msg) {
    {
      std::lock_guard<std::mutex> g(mu);
      if (fired.load()) return;
      why = msg;
      fired.store(1);
    }
    std::fprintf(stderr, "[lwaaai] communicator watchdog: %s\n", msg.c_str());
    std::fflush(stderr);
    if (action == 0) {
      if (comm != nullptr) ncclCommAbort(comm);
      std::fprintf(stderr, "[lwaaai] communicator aborted; exiting with code 86\n");
      std::fflush(stderr);
      _exit(86);
    }
  }

  void loop() {
    (void)hipSetDevice(device);
    const auto period = std::chrono::milliseconds(
        (int)std::max(10.0, std::min(500.0, timeout_s * 1000.0 / 20.0)));
    while (!stop.load() && !fired.load()) {
      std::this_thread::sleep_for(period);
      if (comm != nullptr) {
        ncclResult_t r = ncclSuccess;
        if (ncclCommGetAsyncError(comm, &r) == ncclSuccess && r != ncclSuccess &&
            r != ncclInProgress) {
          fail(std::string("RCCL asynchronous error: ") + ncclGetErrorString(r));
          break;
        }
      }
      std::unique_lock<std::mutex> g(mu);
      if (!pending) continue;
      const hipError_t q = hipEventQuery(ev);
      if (q == hipSuccess) {
        pending = false;
      } else if (q == hipErrorNotReady) {
        const double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() -
                                                            t_mark).count();
        if (waited > timeout_s) {
          g.unlock();
          fail("training step not complete " + std::to_string(waited) + " s after it was " +
               "enqueued (deadline " + std::to_string(timeout_s) + " s): a peer rank is not " +
               "taking part in the collectives");
          break;
        }
      } else {
        g.unlock();
        fail(std::string("device error while waiting for the step: ") + hipGetErrorString(q));
        break;
      }
    }
  }
};

int64_t rccl_watch_start(int64_t h, double timeout_s, int64_t action, int64_t device) {
  auto* w = new Watchdog();
  w->comm = h != 0 ? comm_of(h) : nullptr;
  w->device = (int)device;
  w->timeout_s = timeout_s;
  w->action = (int)action;
  const c10::DeviceGuard guard(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  TORCH_CHECK(hipEventCreateWithFlags(&w->ev, hipEventDisableTiming) == hipSuccess,
              "watchdog: hipEventCreate failed");
  w->th = std::thread([w] { w->loop(); });
  return reinterpret_cast<int64_t>(w);
}

Watchdog* watch_of(int64_t wh) {
  TORCH_CHECK(wh != 0, "watchdog not started");
  return reinterpret_cast<Watchdog*>(wh);
}

// Record the step's completion event on the current stream (skipped while capturing).
void rccl_watch_mark(int64_t wh) {
  Watchdog* w = watch_of(wh);
  hipStream_t st = cur_stream();
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) return;
  std::lock_guard<std::mutex> g(w->mu);
  if (w->pending) {
    // keep the older deadline running until that step completes
    if (hipEventQuery(w->ev) != hipSuccess) return;
    w->pending = false;
  }
  TORCH_CHECK(hipEventRecord(w->ev, st) == hipSuccess, "watchdog: hipEventRecord failed");
  w->t_mark = std::chrono::steady_clock::now();
  w->pending = true;
}

// "" while healthy, else the failure reason (action 1 watchdogs).
std::string rccl_watch_status(int64_t wh) {
  Watchdog* w = watch_of(wh);
  if (!w->fired.load()) return std::string();
  std::lock_guard<std::mutex> g(w->mu);
  return w->why;
}

void rccl_watch_stop(int64_t wh) {
  if (wh == 0) return;
  Watchdog* w = watch_of(wh);
  w->stop.store(true);
  if (w->th.joinable()) w->th.join();
  if (w->ev != nullptr) (void)hipEventDestroy(w->ev);
  delete w;
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(lwaaai, m) {
  m.def("rccl_watch_start(int comm, float timeout_s, int action, int device) -> int",
        &rccl_watch_start);
  m.def("rccl_watch_mark(int watch) -> ()", &rccl_watch_mark);
  m.def("rccl_watch_status(int watch) -> str", &rccl_watch_status);
  m.def("rccl_watch_stop(int watch) -> ()", &rccl_watch_stop);
  m.def("rccl_unique_id() -> Tensor", &rccl_unique_id);
  m.def("rccl_init(Tensor uid, int world, int rank, int device, float timeout_s) -> int",
        &rccl_init);
  m.def("rccl_destroy(int comm) -> ()", &rccl_destroy);
  m.def("rccl_abort(int comm) -> ()", &rccl_abort);
  m.def("rccl_all_gather(int comm, Tensor send, Tensor(a!) recv) -> ()", &rccl_all_gather);
  m.def("rccl_all_reduce(int comm, Tensor(a!) t, int op) -> ()", &rccl_all_reduce);
  m.def("rccl_broadcast(int comm, Tensor(a!) t, int root) -> ()", &rccl_broadcast);
  m.def("rccl_send_recv(int comm, Tensor[] sends, int[] send_peers, Tensor(a!)[] recvs, "
        "int[] recv_peers) -> ()", &rccl_send_recv);
  m.def("rccl_all_to_all(int comm, Tensor send, Tensor(a!) recv) -> ()", &rccl_all_to_all);
  m.def("rccl_reduce_scatter(int comm, Tensor send, Tensor(a!) recv, int op) -> ()",
        &rccl_reduce_scatter);
}
