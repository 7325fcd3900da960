// torch op bindings for the layer_wise_aaai20_amd HIP kernels (namespace torch.ops.lwaaai).
//
// Registered through the dispatcher for the CUDA key (= HIP on ROCm builds of PyTorch); there is
// deliberately NO CPU kernel here: CPU tensors use the pure-torch implementation in
// layer_wise_aaai20_amd/ops, and a GPU tensor reaching an op without this library loaded fails
// loudly in ops/_ext.py.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPCachingAllocatorMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>
#include <map>
#include <mutex>
#include <torch/library.h>

#include <algorithm>

#include "lw_kernels.h"

// The 16-bit element of the fused path (elem16.h): bf16 in lwaaai, fp16 in the lwaaai16 build of
// the same sources (csrc/build.py), whose ops register under torch.ops.lwaaai16.
#ifndef LW_OPS_NS
#define LW_OPS_NS lwaaai
#endif
#ifdef LW_FP16
#define LW_H16_TYPE at::kHalf
#else
#define LW_H16_TYPE at::kBFloat16
#endif
// one expansion step so that TORCH_LIBRARY pastes the namespace's value, not the macro name
#define LW_LIBRARY(ns, m) TORCH_LIBRARY(ns, m)
#define LW_LIBRARY_IMPL(ns, k, m) TORCH_LIBRARY_IMPL(ns, k, m)

namespace {

using at::Tensor;
constexpr at::ScalarType kH16 = LW_H16_TYPE;

// ROCm builds of PyTorch expose HIP devices as DeviceType::CUDA ("masquerading").
inline hipStream_t cur_stream() {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
}

template <typename T>
inline T* ptr(const Tensor& t) { return reinterpret_cast<T*>(t.data_ptr()); }
template <typename T>
inline T* optr(const c10::optional<Tensor>& t) {
  return (t.has_value() && t->defined()) ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

// Every binding checks its launches: a bad launch configuration (or a failed async memset before
// it) raises here, at the op that caused it, instead of surfacing later or not at all.
// BN kernels keep one 8-channel group per thread of a 256-thread block (bn.hip)
constexpr int64_t kMaxBnC = 8 * 256;

void launched(const char* op) {
  const hipError_t e = hipGetLastError();
  TORCH_CHECK(e == hipSuccess, "HIP launch failed in lwaaai.", op, ": ", hipGetErrorString(e));
}

void check_cuda(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
void check_dtype(const Tensor& t, at::ScalarType st, const char* name) {
  TORCH_CHECK(t.scalar_type() == st, name, " has dtype ", t.scalar_type(), ", expected ", st);
}
void check_aligned16(const void* p, const char* name) {
  TORCH_CHECK((reinterpret_cast<uintptr_t>(p) & 15u) == 0, name, " must be 16-byte aligned");
}

// Scratch layout shared by all selection ops (one workspace tensor per bucket plan, reused).
struct Carve {
  int64_t off = 0;
  template <typename T>
  int64_t take(int64_t n) {
    const int64_t o = off;
    off += ((int64_t)sizeof(T) * std::max<int64_t>(n, 1) + 255) / 256 * 256;
    return o;
  }
};
struct WsLayout {
  int64_t hist, st_small, st_large, cnt, pre, partial, segmax, total;
};
WsLayout layout(int64_t n_small, int64_t n_large, int64_t n_tasks) {
  Carve c;
  WsLayout w;
  w.hist = c.take<uint32_t>(n_large * 4096);
  w.st_small = c.take<lw::SelState>(n_small);
  w.st_large = c.take<lw::SelState>(n_large);
  // (per quarter task: the fused select chain counts and writes 2048-element sub-tasks)
  w.cnt = c.take<uint2>(n_tasks * lw::kWriteSub);
  w.pre = c.take<uint2>(n_tasks * lw::kWriteSub);
  w.partial = c.take<float2>(n_tasks);
  w.segmax = c.take<float>(n_large);
  w.total = c.off;
  return w;
}

int64_t workspace_bytes(int64_t n_small, int64_t n_large, int64_t n_tasks) {
  return layout(n_small, n_large, n_tasks).total;
}

// optional device step counter (int32/int64 scalar; the kernels read its low 32 bits)
const uint32_t* step_ptr(const c10::optional<Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  check_cuda(*t, "step_t");
  TORCH_CHECK((t->scalar_type() == at::kInt || t->scalar_type() == at::kLong) && t->numel() >= 1,
              "step_t must be an int32/int64 GPU scalar");
  return reinterpret_cast<const uint32_t*>(t->data_ptr());
}

// optional device overflow counter (int64 scalar, incremented with 64-bit atomics: a 32-bit
// count of capped threshold hits wraps within a few hundred steps)
unsigned long long* overflow_ptr(const c10::optional<Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  check_cuda(*t, "overflow");
  TORCH_CHECK(t->scalar_type() == at::kLong && t->numel() >= 1,
              "overflow must be an int64 GPU tensor");
  return reinterpret_cast<unsigned long long*>(t->data_ptr());
}

lw::SelectArgs make_select_args(const Tensor& g, const c10::optional<Tensor>& ef,
                                const Tensor& seg_off, const Tensor& seg_n, const Tensor& keep,
                                const Tensor& cap_off, const Tensor& small_segs,
                                const Tensor& large_segs, const Tensor& tasks,
                                const Tensor& task_lo, const Tensor& ws) {
  check_cuda(g, "g");
  check_dtype(g, at::kFloat, "g");
  check_aligned16(g.data_ptr(), "g");
  check_dtype(seg_off, at::kLong, "seg_off");
  check_dtype(cap_off, at::kLong, "cap_off");
  check_dtype(seg_n, at::kInt, "seg_n");
  check_dtype(keep, at::kInt, "keep");
  check_dtype(tasks, at::kInt, "tasks");
  if (ef.has_value() && ef->defined()) {
    check_cuda(*ef, "ef");
    check_dtype(*ef, at::kFloat, "ef");
    TORCH_CHECK(ef->numel() >= g.numel(), "ef smaller than g");
    check_aligned16(ef->data_ptr(), "ef");
  }
  lw::SelectArgs a{};
  a.g = ptr<float>(g);
  a.ef = optr<float>(ef);
  a.seg_off = ptr<int64_t>(seg_off);
  a.seg_n = ptr<int32_t>(seg_n);
  a.keep = ptr<int32_t>(keep);
  a.cap_off = ptr<int64_t>(cap_off);
  a.small_segs = ptr<int32_t>(small_segs);
  a.large_segs = ptr<int32_t>(large_segs);
  a.tasks = ptr<int2>(tasks);
  a.task_lo = ptr<int32_t>(task_lo);
  a.n_small = (int)small_segs.numel();
  a.n_large = (int)large_segs.numel();
  a.n_tasks = (int)(tasks.numel() / 2);
  const WsLayout L = layout(a.n_small, a.n_large, a.n_tasks);
  TORCH_CHECK(ws.numel() >= L.total, "workspace too small: ", ws.numel(), " < ", L.total);
  uint8_t* base = ptr<uint8_t>(ws);
  a.hist = reinterpret_cast<uint32_t*>(base + L.hist);
  a.st_small = reinterpret_cast<lw::SelState*>(base + L.st_small);
  a.st_large = reinterpret_cast<lw::SelState*>(base + L.st_large);
  a.cnt = reinterpret_cast<uint2*>(base + L.cnt);
  a.pre = reinterpret_cast<uint2*>(base + L.pre);
  return a;
}

void select_compress(Tensor g, c10::optional<Tensor> ef, Tensor seg_off, Tensor seg_n,
                     Tensor keep, Tensor cap_off, Tensor small_segs, Tensor large_segs,
                     Tensor tasks, Tensor task_lo, Tensor ws, int64_t km, int64_t out,
                     c10::optional<Tensor> pairs, c10::optional<Tensor> vals,
                     c10::optional<Tensor> idx, int64_t gid_base, int64_t step, int64_t seed,
                     c10::optional<Tensor> step_t, c10::optional<Tensor> overflow,
                     c10::optional<Tensor> mom, bool staged, int64_t max_seg_tasks,
                     c10::optional<Tensor> mc_p, c10::optional<Tensor> mc_wd, double mc,
                     double mc_wmul) {
  const c10::DeviceGuard guard(g.device());
  lw::SelectArgs a = make_select_args(g, ef, seg_off, seg_n, keep, cap_off, small_segs, large_segs,
                                      tasks, task_lo, ws);
  a.max_seg_tasks = (int)max_seg_tasks;
  if (mom.has_value() && mom->defined()) {
    check_cuda(*mom, "mom");
    check_dtype(*mom, at::kFloat, "mom");
    TORCH_CHECK(mom->numel() >= g.numel() && mom->is_contiguous(), "mom: g's layout");
    a.mom = ptr<float>(*mom);
  }
  a.pairs = optr<int2>(pairs);
  a.vals = optr<float>(vals);
  a.idx_out = optr<int32_t>(idx);
  TORCH_CHECK(out == lw::OUT_PAIRS ? a.pairs != nullptr : (a.vals && a.idx_out),
              "missing output buffers");
  if (mc != 0.0) {                 // momentum correction fused into the first pass (McArgs)
    TORCH_CHECK(a.mom != nullptr, "select_compress: fused momentum correction needs mom (u)");
    TORCH_CHECK(km == lw::KM_TOPK && out == lw::OUT_PAIRS && !staged,
                "select_compress: fused momentum correction is Top-K pairs, unstaged");
    a.mcx.u = a.mom;
    a.mcx.mc = (float)mc;
    a.mcx.wmul = (float)mc_wmul;
    if (mc_wd.has_value() && mc_wd->defined() && mc_p.has_value() && mc_p->defined()) {
      check_cuda(*mc_p, "mc_p");
      check_dtype(*mc_p, at::kFloat, "mc_p");
      check_dtype(*mc_wd, at::kFloat, "mc_wd");
      TORCH_CHECK(mc_p->is_contiguous() && mc_p->numel() >= g.numel(), "mc_p: g's layout");
      check_aligned16(mc_p->data_ptr(), "mc_p");
      a.mcx.p = ptr<float>(*mc_p);
      a.mcx.wd = ptr<float>(*mc_wd);
    }
  }
  a.gid_base = (uint32_t)gid_base;
  a.step = (uint32_t)step;
  a.step_ptr = step_ptr(step_t);
  a.overflow = overflow_ptr(overflow);
  a.seed0 = (uint32_t)(seed & 0xffffffff);
  a.seed1 = (uint32_t)((uint64_t)seed >> 32);
  lw::select_compress(a, (int)km, (int)out, a.ef != nullptr, cur_stream(), staged);
  launched("select_compress");
}

// entire-model staging (compress.hip select_stage): pass 0 over tasks [t_lo, t_hi)
void select_stage(Tensor g, c10::optional<Tensor> ef, Tensor seg_off, Tensor seg_n, Tensor keep,
                  Tensor cap_off, Tensor small_segs, Tensor large_segs, Tensor tasks,
                  Tensor task_lo, Tensor ws, int64_t km, int64_t t_lo, int64_t t_hi, bool zero,
                  int64_t gid_base, int64_t step, int64_t seed, c10::optional<Tensor> step_t) {
  const c10::DeviceGuard guard(g.device());
  lw::SelectArgs a = make_select_args(g, ef, seg_off, seg_n, keep, cap_off, small_segs, large_segs,
                                      tasks, task_lo, ws);
  TORCH_CHECK(0 <= t_lo && t_lo <= t_hi && t_hi <= a.n_tasks, "select_stage: task range");
  TORCH_CHECK(km == lw::KM_TOPK || km == lw::KM_RANDK, "select_stage: Top-K / Random-K");
  a.gid_base = (uint32_t)gid_base;
  a.step = (uint32_t)step;
  a.step_ptr = step_ptr(step_t);
  a.seed0 = (uint32_t)(seed & 0xffffffff);
  a.seed1 = (uint32_t)((uint64_t)seed >> 32);
  // (one entire-model segment: this stage's tasks all add into its one histogram)
  a.max_seg_tasks = a.n_large == 1 ? (int)(t_hi - t_lo) : 0;
  lw::select_stage(a, (int)km, a.ef != nullptr, (int)t_lo, (int)t_hi, zero, cur_stream());
  launched("select_stage");
}

void thresh_count(Tensor g, c10::optional<Tensor> ef, Tensor seg_off, Tensor seg_n,
                  Tensor large_segs, Tensor tasks, Tensor task_lo, Tensor ws, double V,
                  int64_t adaptive, Tensor counts_out) {
  const c10::DeviceGuard guard(g.device());
  Tensor empty_i = at::empty({0}, seg_n.options());
  Tensor empty_l = at::empty({1}, seg_off.options());
  lw::SelectArgs a = make_select_args(g, ef, seg_off, seg_n, seg_n, empty_l.expand({2}).contiguous(),
                                      empty_i, large_segs, tasks, task_lo, ws);
  check_dtype(counts_out, at::kInt, "counts_out");
  const WsLayout L = layout(a.n_small, a.n_large, a.n_tasks);
  uint8_t* base = ptr<uint8_t>(ws);
  lw::thresh_count(a, (float)V, (int)adaptive, a.ef != nullptr,
                   reinterpret_cast<float*>(base + L.segmax),
                   reinterpret_cast<float2*>(base + L.partial), ptr<int32_t>(counts_out),
                   cur_stream());
  launched("thresh_count");
}

void thresh_dense(Tensor g, c10::optional<Tensor> ef, Tensor seg_off, Tensor seg_n,
                  Tensor large_segs, Tensor tasks, Tensor task_lo, Tensor ws, double V,
                  int64_t adaptive) {
  const c10::DeviceGuard guard(g.device());
  Tensor empty_i = at::empty({0}, seg_n.options());
  Tensor empty_l = at::empty({1}, seg_off.options());
  lw::SelectArgs a = make_select_args(g, ef, seg_off, seg_n, seg_n, empty_l.expand({2}).contiguous(),
                                      empty_i, large_segs, tasks, task_lo, ws);
  const WsLayout L = layout(a.n_small, a.n_large, a.n_tasks);
  uint8_t* base = ptr<uint8_t>(ws);
  lw::thresh_dense(a, (float)V, (int)adaptive, a.ef != nullptr,
                   reinterpret_cast<float*>(base + L.segmax),
                   reinterpret_cast<float2*>(base + L.partial), cur_stream());
  launched("thresh_dense");
}

void thresh_write(Tensor g, c10::optional<Tensor> ef, Tensor seg_off, Tensor seg_n,
                  Tensor cap_off, Tensor large_segs, Tensor tasks, Tensor task_lo, Tensor ws,
                  Tensor pairs, c10::optional<Tensor> overflow) {
  const c10::DeviceGuard guard(g.device());
  Tensor empty_i = at::empty({0}, seg_n.options());
  lw::SelectArgs a = make_select_args(g, ef, seg_off, seg_n, seg_n, cap_off, empty_i, large_segs,
                                      tasks, task_lo, ws);
  check_cuda(pairs, "pairs");
  a.pairs = ptr<int2>(pairs);
  a.overflow = overflow_ptr(overflow);
  lw::thresh_write(a, a.ef != nullptr, cur_stream());
  launched("thresh_write");
}

void unpack_pairs(Tensor gathered, int64_t world, Tensor g, Tensor seg_off, Tensor seg_n,
                  Tensor cap_off, Tensor utasks) {
  const c10::DeviceGuard guard(g.device());
  check_cuda(gathered, "gathered");
  check_cuda(g, "g");
  check_aligned16(g.data_ptr(), "g");
  TORCH_CHECK(world >= 1 && world <= lw::kMaxWorld, "world size out of range");
  const int64_t cap_total = gathered.numel() / 2 / world;
  lw::unpack_pairs(ptr<int2>(gathered), cap_total, (int)world, ptr<float>(g), ptr<int64_t>(seg_off),
                   ptr<int32_t>(seg_n), ptr<int64_t>(cap_off), ptr<int2>(utasks),
                   (int)(utasks.numel() / 2), cur_stream());
  launched("unpack_pairs");
}

// decode of a layer-wise Top-K bucket fused with its SGD step (compress.hip k_unpack_sgd): p, buf,
// pb are the bucket's slices of the parameter / momentum / bf16-mirror arenas, seg_wd the decay of
// its segments
void unpack_pairs_sgd(Tensor gathered, int64_t world, Tensor seg_off, Tensor cap_off,
                      Tensor ftasks, Tensor p, Tensor buf, Tensor seg_wd,
                      double lr, double momentum, double dampening, int64_t nesterov,
                      int64_t first_step, double grad_scale, c10::optional<Tensor> hyper,
                      c10::optional<Tensor> pb) {
  const c10::DeviceGuard guard(p.device());
  check_cuda(gathered, "gathered");
  check_cuda(p, "p");
  check_dtype(p, at::kFloat, "p");
  check_dtype(seg_wd, at::kFloat, "seg_wd");
  TORCH_CHECK(world >= 1 && world <= lw::kMaxWorld, "world size out of range");
  TORCH_CHECK(p.is_contiguous() && seg_wd.is_contiguous(), "unpack_pairs_sgd: contiguous p");
  lw::SgdArgs a{};
  a.p = ptr<float>(p);
  a.g = nullptr;
  a.buf = nullptr;
  if (momentum != 0.0) {
    check_cuda(buf, "buf");
    TORCH_CHECK(buf.scalar_type() == at::kFloat && buf.numel() == p.numel() && buf.is_contiguous(),
                "unpack_pairs_sgd: momentum slice must match p");
    a.buf = ptr<float>(buf);
  }
  a.seg_wd = ptr<float>(seg_wd);
  a.lr = (float)lr;
  a.momentum = (float)momentum;
  a.dampening = (float)dampening;
  a.grad_scale = (float)grad_scale;
  a.nesterov = (int)nesterov;
  a.first_step = (int)first_step;
  if (hyper.has_value() && hyper->defined()) {
    check_cuda(*hyper, "hyper");
    TORCH_CHECK(hyper->scalar_type() == at::kFloat && hyper->numel() >= 2 &&
                    hyper->is_contiguous(), "hyper must be a contiguous float32 [lr, grad_scale]");
    a.hyper = hyper->data_ptr<float>();
  }
  if (pb.has_value() && pb->defined()) {
    check_cuda(*pb, "pb");
    TORCH_CHECK(pb->scalar_type() == kH16 && pb->numel() == p.numel() && pb->is_contiguous(),
                "pb must be a 16-bit tensor with p's layout");
    a.pb = reinterpret_cast<uint16_t*>(pb->data_ptr());
  }
  const int64_t cap_total = gathered.numel() / 2 / world;
  check_cuda(ftasks, "ftasks");
  check_dtype(ftasks, at::kInt, "ftasks");
  TORCH_CHECK(ftasks.dim() == 2 && ftasks.size(1) == 4 && ftasks.is_contiguous(),
              "unpack_pairs_sgd: ftasks must be a contiguous [T, 4] int32 table");
  lw::unpack_pairs_sgd(ptr<int2>(gathered), cap_total, (int)world, ptr<int64_t>(seg_off),
                       ptr<int64_t>(cap_off), reinterpret_cast<const int4*>(ftasks.data_ptr()),
                       (int)ftasks.size(0), a, cur_stream());
  launched("unpack_pairs_sgd");
}

void unpack_validx(Tensor vals, Tensor idx, Tensor slot_seg, int64_t world, Tensor g,
                   Tensor seg_off) {
  const c10::DeviceGuard guard(g.device());
  check_cuda(vals, "vals");
  check_cuda(g, "g");
  lw::unpack_validx(ptr<float>(vals), ptr<int32_t>(idx), ptr<int32_t>(slot_seg), vals.numel(),
                    (int)world, ptr<float>(g), ptr<int64_t>(seg_off), cur_stream());
  launched("unpack_validx");
}

lw::QuantArgs make_quant_args(const Tensor& g, const c10::optional<Tensor>& ef,
                              const Tensor& seg_off, const Tensor& seg_n, const Tensor& segs,
                              const Tensor& tasks, const Tensor& task_lo, const Tensor& rec_off,
                              int64_t qstates) {
  check_cuda(g, "g");
  check_dtype(g, at::kFloat, "g");
  check_aligned16(g.data_ptr(), "g");
  lw::QuantArgs a{};
  a.g = ptr<float>(g);
  a.ef = optr<float>(ef);
  a.seg_off = ptr<int64_t>(seg_off);
  a.seg_n = ptr<int32_t>(seg_n);
  a.segs = ptr<int32_t>(segs);
  a.tasks = ptr<int2>(tasks);
  a.task_lo = ptr<int32_t>(task_lo);
  a.rec_off = ptr<int64_t>(rec_off);
  a.nseg = (int)segs.numel();
  a.n_tasks = (int)(tasks.numel() / 2);
  a.qstates = (int)qstates;
  return a;
}

void quantize(Tensor g, c10::optional<Tensor> ef, Tensor seg_off, Tensor seg_n, Tensor segs,
              Tensor tasks, Tensor task_lo, Tensor rec_off, Tensor ws, Tensor payload, int64_t q,
              int64_t qstates, int64_t gid_base, int64_t step, int64_t tag, int64_t seed,
              c10::optional<Tensor> step_t, bool staged) {
  const c10::DeviceGuard guard(g.device());
  lw::QuantArgs a = make_quant_args(g, ef, seg_off, seg_n, segs, tasks, task_lo, rec_off, qstates);
  check_cuda(payload, "payload");
  check_aligned16(payload.data_ptr(), "payload");
  const WsLayout L = layout(0, a.nseg, a.n_tasks);
  TORCH_CHECK(ws.numel() >= L.total, "workspace too small");
  uint8_t* base = ptr<uint8_t>(ws);
  a.scale = reinterpret_cast<float*>(base + L.segmax);
  a.payload = ptr<uint32_t>(payload);
  a.gid_base = (uint32_t)gid_base;
  a.step = (uint32_t)step;
  a.step_ptr = step_ptr(step_t);
  a.tag = (uint32_t)tag;
  a.seed0 = (uint32_t)(seed & 0xffffffff);
  a.seed1 = (uint32_t)((uint64_t)seed >> 32);
  lw::seg_reduce(a, a.ef != nullptr, q == lw::Q_TERN ? 0 : 1, a.scale,
                 reinterpret_cast<float2*>(base + L.partial), cur_stream(), staged);
  launched("seg_reduce");
  // after seg_reduce the EF add is already folded into g (g' = g + e)
  lw::quantize(a, (int)q, a.ef != nullptr, cur_stream());
  launched("quantize");
}

// entire-model staging of the quantisers (compress.hip quant_stage)
void quant_stage(Tensor g, c10::optional<Tensor> ef, Tensor seg_off, Tensor seg_n, Tensor segs,
                 Tensor tasks, Tensor task_lo, Tensor rec_off, Tensor ws, int64_t qstates,
                 int64_t t_lo, int64_t t_hi) {
  const c10::DeviceGuard guard(g.device());
  lw::QuantArgs a = make_quant_args(g, ef, seg_off, seg_n, segs, tasks, task_lo, rec_off, qstates);
  TORCH_CHECK(0 <= t_lo && t_lo <= t_hi && t_hi <= a.n_tasks, "quant_stage: task range");
  const WsLayout L = layout(0, a.nseg, a.n_tasks);
  TORCH_CHECK(ws.numel() >= L.total, "workspace too small");
  uint8_t* base = ptr<uint8_t>(ws);
  lw::quant_stage(a, a.ef != nullptr, (int)t_lo, (int)t_hi,
                  reinterpret_cast<float2*>(base + L.partial), cur_stream());
  launched("quant_stage");
}

void dequantize(Tensor gathered, int64_t world, Tensor g, Tensor seg_off, Tensor seg_n,
                Tensor segs, Tensor tasks, Tensor task_lo, Tensor rec_off, int64_t q,
                int64_t qstates) {
  const c10::DeviceGuard guard(g.device());
  lw::QuantArgs a = make_quant_args(g, c10::nullopt, seg_off, seg_n, segs, tasks, task_lo, rec_off,
                                    qstates);
  check_cuda(gathered, "gathered");
  check_aligned16(gathered.data_ptr(), "gathered");
  const int64_t wpr = gathered.numel() / world;
  TORCH_CHECK(wpr % 4 == 0, "payload words per rank must be a multiple of 4");
  lw::dequantize(a, (int)q, ptr<uint32_t>(gathered), wpr, (int)world, cur_stream());
  launched("dequantize");
}

// quantised reduce-scatter wire (compress.hip k_dequant_shard, k_bf16_expand)
void dequant_shard(Tensor recv, int64_t world, int64_t hdr, Tensor gtab, int64_t g0, int64_t ng,
                   int64_t q, int64_t qstates, Tensor out) {
  const c10::DeviceGuard guard(out.device());
  check_cuda(recv, "recv");
  check_cuda(gtab, "gtab");
  check_cuda(out, "out");
  check_dtype(recv, at::kInt, "recv");
  check_dtype(gtab, at::kInt, "gtab");
  check_dtype(out, at::kBFloat16, "out");
  check_aligned16(recv.data_ptr(), "recv");
  check_aligned16(out.data_ptr(), "out");
  TORCH_CHECK(world >= 1 && recv.numel() % world == 0, "dequant_shard: recv must hold world pieces");
  const int64_t wpr = recv.numel() / world;
  const int64_t rl = q == 0 ? 2 : (q == 3 ? 16 : 8);
  TORCH_CHECK(wpr % 4 == 0 && hdr % 4 == 0, "dequant_shard: pieces must be 16-byte multiples");
  TORCH_CHECK(wpr >= hdr + ng * rl + (q == 2 ? ng : 0), "dequant_shard: pieces too small");
  TORCH_CHECK(gtab.dim() == 2 && gtab.size(1) == 4 && g0 >= 0 && g0 + ng <= gtab.size(0),
              "dequant_shard: group table [G][4] does not cover the shard");
  lw::dequantize_shard((int)q, ptr<uint32_t>(recv), wpr, (int)world, (int)hdr,
                       reinterpret_cast<const int4*>(gtab.data_ptr()), g0, ng, (int)qstates,
                       ptr<uint16_t>(out), out.numel(), cur_stream());
  launched("dequant_shard");
}

void wire_wait(Tensor dev, double us, int64_t nwg) {
  const c10::DeviceGuard guard(dev.device());
  TORCH_CHECK(us < 1e6 && nwg >= 0 && nwg <= 1024, "wire_wait: at most 1 s on 1024 workgroups");
  lw::wire_wait(us, (int)nwg, cur_stream());
  launched("wire_wait");
}

void bf16_expand(Tensor in, Tensor out) {
  const c10::DeviceGuard guard(out.device());
  check_cuda(in, "in");
  check_cuda(out, "out");
  check_dtype(in, at::kBFloat16, "in");
  check_dtype(out, at::kFloat, "out");
  TORCH_CHECK(in.numel() == out.numel(), "bf16_expand: size mismatch");
  check_aligned16(in.data_ptr(), "in");
  check_aligned16(out.data_ptr(), "out");
  lw::bf16_expand(ptr<uint16_t>(in), ptr<float>(out), in.numel(), cur_stream());
  launched("bf16_expand");
}

// momentum correction prologue / masking (optim.hip k_mc_prep, k_mc_mask)
void mc_prep(Tensor g, Tensor u, c10::optional<Tensor> p, Tensor seg_off, Tensor seg_n,
             Tensor segs, Tensor tasks, c10::optional<Tensor> seg_wd, double mc, double wmul) {
  const c10::DeviceGuard guard(g.device());
  check_cuda(g, "g");
  check_cuda(u, "u");
  check_dtype(g, at::kFloat, "g");
  check_dtype(u, at::kFloat, "u");
  TORCH_CHECK(g.is_contiguous() && u.is_contiguous() && u.numel() == g.numel(),
              "mc_prep: g and u must be contiguous and of one size");
  check_aligned16(g.data_ptr(), "g");
  check_aligned16(u.data_ptr(), "u");
  const float* pp = nullptr;
  const float* wd = nullptr;
  if (p.has_value() && p->defined() && seg_wd.has_value() && seg_wd->defined()) {
    check_cuda(*p, "p");
    check_dtype(*p, at::kFloat, "p");
    TORCH_CHECK(p->is_contiguous() && p->numel() == g.numel(), "mc_prep: p must have g's layout");
    check_aligned16(p->data_ptr(), "p");
    check_dtype(*seg_wd, at::kFloat, "seg_wd");
    pp = ptr<float>(*p);
    wd = ptr<float>(*seg_wd);
  }
  check_dtype(seg_off, at::kLong, "seg_off");
  check_dtype(seg_n, at::kInt, "seg_n");
  check_dtype(tasks, at::kInt, "tasks");
  lw::mc_prep(ptr<float>(g), ptr<float>(u), pp, ptr<int64_t>(seg_off), ptr<int32_t>(seg_n),
              ptr<int32_t>(segs), ptr<int2>(tasks), (int)(tasks.numel() / 2), wd, (float)mc,
              (float)wmul, cur_stream());
  launched("mc_prep");
}

// the engine's device step counter (+1 per step inside the captured graph; csrc/optim.hip)
void step_bump(Tensor c) {
  const c10::DeviceGuard guard(c.device());
  check_cuda(c, "c");
  check_dtype(c, at::kLong, "c");
  TORCH_CHECK(c.numel() >= 1, "step_bump: empty counter");
  lw::step_bump(ptr<int64_t>(c), cur_stream());
  launched("step_bump");
}

void mc_mask(Tensor u, Tensor e) {
  const c10::DeviceGuard guard(u.device());
  check_cuda(u, "u");
  check_cuda(e, "e");
  check_dtype(u, at::kFloat, "u");
  check_dtype(e, at::kFloat, "e");
  TORCH_CHECK(u.is_contiguous() && e.is_contiguous() && u.numel() == e.numel(),
              "mc_mask: u and e must be contiguous and of one size");
  check_aligned16(u.data_ptr(), "u");
  check_aligned16(e.data_ptr(), "e");
  lw::mc_mask(ptr<float>(u), ptr<float>(e), u.numel(), cur_stream());
  launched("mc_mask");
}

void sgd_step(Tensor p, Tensor g, Tensor buf, Tensor seg_off, Tensor seg_n, Tensor segs,
              Tensor tasks, Tensor seg_wd, double lr, double momentum, double dampening,
              int64_t nesterov, int64_t first_step, double grad_scale,
              c10::optional<Tensor> hyper, c10::optional<Tensor> pb) {
  const c10::DeviceGuard guard(p.device());
  check_cuda(p, "p");
  check_cuda(g, "g");
  check_aligned16(p.data_ptr(), "p");
  check_aligned16(g.data_ptr(), "g");
  lw::SgdArgs a{};
  a.p = ptr<float>(p);
  a.g = ptr<float>(g);
  a.buf = buf.numel() ? ptr<float>(buf) : nullptr;
  if (momentum != 0.0) {
    TORCH_CHECK(buf.numel() >= p.numel(), "momentum buffer too small");
    check_aligned16(buf.data_ptr(), "buf");
  }
  a.seg_off = ptr<int64_t>(seg_off);
  a.seg_n = ptr<int32_t>(seg_n);
  a.segs = ptr<int32_t>(segs);
  a.tasks = ptr<int2>(tasks);
  a.seg_wd = ptr<float>(seg_wd);
  a.n_tasks = (int)(tasks.numel() / 2);
  a.lr = (float)lr;
  a.momentum = (float)momentum;
  a.dampening = (float)dampening;
  a.grad_scale = (float)grad_scale;
  a.nesterov = (int)nesterov;
  a.first_step = (int)first_step;
  if (hyper.has_value() && hyper->defined()) {
    check_cuda(*hyper, "hyper");
    TORCH_CHECK(hyper->scalar_type() == at::kFloat && hyper->numel() >= 2 &&
                    hyper->is_contiguous(), "hyper must be a contiguous float32 [lr, grad_scale]");
    a.hyper = hyper->data_ptr<float>();
  }
  if (pb.has_value() && pb->defined()) {
    check_cuda(*pb, "pb");
    TORCH_CHECK(pb->scalar_type() == kH16 && pb->numel() == p.numel(),
                "pb must be a bf16 tensor with p's layout");
    check_aligned16(pb->data_ptr(), "pb");
    a.pb = reinterpret_cast<uint16_t*>(pb->data_ptr());
  }
  lw::sgd_step(a, cur_stream());
  launched("sgd_step");
}

void cifar_augment(Tensor data, Tensor idx, Tensor prm, int64_t offset, int64_t crop,
                   int64_t cutout, Tensor out) {
  const c10::DeviceGuard guard(data.device());
  check_cuda(data, "data");
  check_cuda(idx, "idx");
  check_cuda(prm, "prm");
  check_dtype(data, at::kFloat, "data");
  check_dtype(idx, at::kLong, "idx");
  check_dtype(prm, at::kInt, "prm");
  TORCH_CHECK(data.dim() == 4 && prm.dim() == 2 && prm.size(1) == 5, "cifar_augment: shapes");
  const int64_t B = idx.numel(), C = data.size(1), Hp = data.size(2), Wp = data.size(3);
  TORCH_CHECK(crop >= 1 && crop <= Hp && crop <= Wp && cutout >= 0 && cutout <= crop,
              "cifar_augment: crop / cutout out of range");
  TORCH_CHECK(offset >= 0 && offset + B <= prm.size(0), "cifar_augment: choice rows out of range");
  // out: [B, C, crop, crop], or [B, 4, crop, crop] for a 3-channel dataset (zero 4th channel)
  TORCH_CHECK(out.is_cuda() && out.dim() == 4 && out.size(0) == B &&
                  (out.size(1) == C || (C == 3 && out.size(1) == 4)) &&
                  out.size(2) == crop && out.size(3) == crop &&
                  out.is_contiguous(at::MemoryFormat::ChannelsLast),
              "cifar_augment: out must be a channels_last [B, C (or 4), crop, crop] GPU tensor");
  TORCH_CHECK(out.scalar_type() == at::kFloat || out.scalar_type() == kH16,
              "cifar_augment: out must be float32 or bfloat16");
  lw::cifar_augment(ptr<float>(data), ptr<int64_t>(idx), ptr<int32_t>(prm), out.data_ptr(),
                    (int)B, (int)C, (int)Hp, (int)Wp, (int)crop, (int)cutout, offset,
                    out.scalar_type() == kH16, cur_stream(), (int)out.size(1));
  launched("cifar_augment");
}

void normalize_u8(Tensor in, Tensor out, std::vector<double> mean, std::vector<double> stdv) {
  const c10::DeviceGuard guard(in.device());
  check_cuda(in, "in");
  check_dtype(in, at::kByte, "in");
  TORCH_CHECK(mean.size() == 3 && stdv.size() == 3, "mean/std need 3 channels");
  TORCH_CHECK(out.scalar_type() == kH16 || out.scalar_type() == at::kFloat,
              "out must be bf16 or fp32");
  // `out` is an NCHW tensor in channels_last memory == the NHWC byte order of `in`
  TORCH_CHECK(out.dim() == 4 && out.is_contiguous(at::MemoryFormat::ChannelsLast),
              "out must be a channels_last NCHW tensor");
  check_aligned16(in.data_ptr(), "in");
  check_aligned16(out.data_ptr(), "out");
  const float m[3] = {(float)mean[0], (float)mean[1], (float)mean[2]};
  const float s[3] = {(float)stdv[0], (float)stdv[1], (float)stdv[2]};
  if (out.size(1) == 4) {                    // 4-channel (zero-padded) bf16 stem input
    TORCH_CHECK(out.scalar_type() == kH16 && out.numel() / 4 * 3 == in.numel() &&
                out.numel() % 4 == 0, "4-channel out: bf16 with in.numel()/3 pixels");
    lw::normalize_u8_c4(ptr<uint8_t>(in), ptr<uint16_t>(out), in.numel() / 3, m, s, cur_stream());
    launched("normalize_u8_c4");
    return;
  }
  TORCH_CHECK(out.numel() == in.numel(), "out/in size mismatch");
  lw::normalize_u8(ptr<uint8_t>(in), out.data_ptr(), in.numel(), m, s,
                   out.scalar_type() == kH16, cur_stream());
  launched("normalize_u8");
}

// global average pool (nn.hip): x channels_last bf16 [N, C, H, W] -> [N, C] bf16
// w [..., R] contiguous 16-bit -> [...] = Σ over the last dim (fp32 sum, 16-bit out)
// out.view(-1, R)[i, :] (=|+=) g[i] (nn.hip k_repeat_store): fp32 g [n], out [n * R] in place
void repeat_store(Tensor g, Tensor out, int64_t R, bool accumulate) {
  const c10::DeviceGuard guard(out.device());
  check_cuda(g, "g");
  check_cuda(out, "out");
  check_dtype(g, at::kFloat, "g");
  check_dtype(out, at::kFloat, "out");
  TORCH_CHECK(g.is_contiguous() && out.is_contiguous() && R >= 1 &&
                  out.numel() == g.numel() * R, "repeat_store: out must be contiguous [n * R]");
  check_aligned16(out.data_ptr(), "out");
  if (out.numel() > 0)
    lw::repeat_store(ptr<float>(g), ptr<float>(out), out.numel(), (int)R, accumulate,
                     cur_stream());
  launched("repeat_store");
}

Tensor sum_repeats(Tensor w, int64_t R) {
  const c10::DeviceGuard guard(w.device());
  TORCH_CHECK(w.is_cuda() && w.is_contiguous(), "sum_repeats: contiguous GPU tensor");
  check_dtype(w, kH16, "w");
  TORCH_CHECK(R >= 1 && R <= 64 && w.numel() % R == 0, "sum_repeats: 1 <= R <= 64 dividing numel");
  const int64_t n = w.numel() / R;
  Tensor out = at::empty({n}, w.options());
  if (n > 0) lw::sum_repeats(ptr<uint16_t>(w), ptr<uint16_t>(out), n, (int)R, cur_stream());
  launched("sum_repeats");
  return out;
}

Tensor gap_fwd(Tensor x) {
  const c10::DeviceGuard guard(x.device());
  TORCH_CHECK(x.is_cuda(), "x must be a GPU tensor");
  check_dtype(x, kH16, "x");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "x must be a channels_last NCHW tensor");
  const int64_t N = x.size(0), C = x.size(1), HW = x.size(2) * x.size(3);
  TORCH_CHECK(C % 8 == 0 && N * C < (1LL << 31) && N * HW * C < (1LL << 34), "gap_fwd: C % 8 == 0");
  check_aligned16(x.data_ptr(), "x");
  Tensor y = at::empty({N, C}, x.options());
  lw::gap_fwd(ptr<uint16_t>(x), ptr<uint16_t>(y), (int)N, (int)HW, (int)C, cur_stream());
  launched("gap_fwd");
  return y;
}

// fused cross-entropy (nn.hip): logits fp32 [B, C] contiguous, target int64 [B] ->
// (loss rows [B], correct [B, 2] (top-1, top-5), grad [B, C] = (softmax - onehot)·gscale or empty)
std::tuple<Tensor, Tensor, Tensor> xent(Tensor logits, Tensor target, double gscale,
                                        int64_t ignore_index, bool want_grad) {
  const c10::DeviceGuard guard(logits.device());
  TORCH_CHECK(logits.is_cuda(), "logits must be a GPU tensor");
  check_dtype(logits, at::kFloat, "logits");
  check_cuda(target, "target");
  check_dtype(target, at::kLong, "target");
  TORCH_CHECK(logits.dim() == 2 && logits.is_contiguous(), "logits must be contiguous [B, C]");
  const int64_t B = logits.size(0), C = logits.size(1);
  TORCH_CHECK(target.dim() == 1 && target.size(0) == B && target.is_contiguous(), "target [B]");
  TORCH_CHECK(B < (1LL << 30) && C > 0 && B * C < (1LL << 40), "xent: size");
  Tensor loss = at::empty({B}, logits.options());
  Tensor corr = at::empty({B, 2}, logits.options());
  Tensor grad = want_grad ? at::empty({B, C}, logits.options()) : at::empty({0}, logits.options());
  if (B > 0)
    lw::xent(ptr<float>(logits), ptr<int64_t>(target), (int)B, (int)C, (float)gscale,
             (int)ignore_index, ptr<float>(loss), ptr<float>(corr),
             want_grad ? ptr<float>(grad) : nullptr, cur_stream());
  launched("xent");
  return {loss, corr, grad};
}

// (mean, count) of xent's per-row losses over the non-ignored targets (one launch): a 0-dim loss
// and a [1] count
std::tuple<Tensor, Tensor> xent_mean(Tensor rows, Tensor target, int64_t ignore_index) {
  const c10::DeviceGuard guard(rows.device());
  check_cuda(rows, "rows");
  check_dtype(rows, at::kFloat, "rows");
  check_cuda(target, "target");
  check_dtype(target, at::kLong, "target");
  TORCH_CHECK(rows.dim() == 1 && target.dim() == 1 && rows.size(0) == target.size(0) &&
              rows.size(0) < (1LL << 30), "xent_mean: rows / target [B]");
  Tensor out = at::empty({}, rows.options());
  Tensor n = at::empty({1}, rows.options());
  lw::xent_mean(ptr<float>(rows), ptr<int64_t>(target), (int)rows.size(0), (int)ignore_index,
                ptr<float>(out), ptr<float>(n), cur_stream());
  launched("xent_mean");
  return {out, n};
}

// grad · (gl / n) with gl, n one-element fp32 device tensors
Tensor xent_scale(Tensor grad, Tensor gl, Tensor n) {
  const c10::DeviceGuard guard(grad.device());
  check_cuda(grad, "grad");
  check_dtype(grad, at::kFloat, "grad");
  check_dtype(gl, at::kFloat, "gl");
  check_dtype(n, at::kFloat, "n");
  TORCH_CHECK(gl.is_cuda() && n.is_cuda() && gl.numel() == 1 && n.numel() >= 1,
              "xent_scale: gl / n device scalars");
  Tensor out = at::empty_like(grad);
  lw::xent_scale(ptr<float>(grad), ptr<float>(gl), ptr<float>(n), grad.numel(), ptr<float>(out),
                 cur_stream());
  launched("xent_scale");
  return out;
}

// bias + ReLU epilogue backward (nn.hip): dy, y bf16 rows [M, C] (channels_last NCHW or 2-D) ->
// (dy·[y > 0] (or dy itself without y), db fp32 [C]; accumulated into db_out when given)
std::tuple<Tensor, Tensor> relu_bias_bwd(Tensor dy, c10::optional<Tensor> y,
                                         c10::optional<Tensor> db_out) {
  const c10::DeviceGuard guard(dy.device());
  TORCH_CHECK(dy.is_cuda(), "dy must be a GPU tensor");
  check_dtype(dy, kH16, "dy");
  const bool cl = dy.dim() == 4 && dy.is_contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(cl || (dy.dim() == 2 && dy.is_contiguous()), "dy: channels_last NCHW or [M, C]");
  const int64_t C = dy.size(1), M = dy.numel() / std::max<int64_t>(C, 1);
  TORCH_CHECK(C % 8 == 0 && C > 0 && (C <= 2048 || C % 2048 == 0) && C <= 16384 &&
              M < (1LL << 40), "relu_bias_bwd: C % 8, <= 2048 or a multiple of 2048");
  check_aligned16(dy.data_ptr(), "dy");
  const bool relu = y.has_value() && y->defined();
  if (relu) {
    check_dtype(*y, kH16, "y");
    TORCH_CHECK(y->sizes() == dy.sizes() && y->strides() == dy.strides(), "y must match dy");
    check_aligned16(y->data_ptr(), "y");
  }
  Tensor dym = relu ? at::empty_like(dy) : dy;
  Tensor db;
  const bool acc = db_out.has_value() && db_out->defined();
  if (acc) {
    db = *db_out;
    check_dtype(db, at::kFloat, "db_out");
    TORCH_CHECK(db.numel() == C && db.is_contiguous(), "db_out [C]");
  } else {
    db = at::empty({C}, dy.options().dtype(at::kFloat));
  }
  Tensor partial = at::empty({(int64_t)lw::relu_bias_bwd_blocks(M, (int)C) * C}, db.options());
  lw::relu_bias_bwd(ptr<uint16_t>(dy), relu ? ptr<uint16_t>(*y) : nullptr,
                    relu ? ptr<uint16_t>(dym) : nullptr, ptr<float>(partial), ptr<float>(db), M,
                    (int)C, acc, cur_stream());
  launched("relu_bias_bwd");
  return {dym, db};
}

// dy [N, C] bf16/fp32 -> channels_last bf16 [N, C, H, W] filled with dy / (H*W)
Tensor gap_bwd(Tensor dy, int64_t H, int64_t W) {
  const c10::DeviceGuard guard(dy.device());
  check_cuda(dy, "dy");
  TORCH_CHECK(dy.dim() == 2 && dy.is_contiguous(), "dy must be a contiguous [N, C] tensor");
  TORCH_CHECK(dy.scalar_type() == kH16 || dy.scalar_type() == at::kFloat,
              "dy must be bf16 or fp32");
  const int64_t N = dy.size(0), C = dy.size(1);
  TORCH_CHECK(C % 8 == 0 && H > 0 && W > 0 && N * H * W * (C / 8) < (1LL << 31),
              "gap_bwd: C % 8 == 0 and N*H*W*C/8 < 2^31");
  check_aligned16(dy.data_ptr(), "dy");
  Tensor dx = at::empty({N, C, H, W}, dy.options().dtype(kH16),
                        at::MemoryFormat::ChannelsLast);
  lw::gap_bwd(dy.data_ptr(), dy.scalar_type() == at::kFloat, ptr<uint16_t>(dx), (int)N,
              (int)(H * W), (int)C, cur_stream());
  launched("gap_bwd");
  return dx;
}

// ---------------------------------------------------------------- fused BatchNorm (NHWC)
void check_nhwc(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.dim() == 4 ? t.is_contiguous(at::MemoryFormat::ChannelsLast) : t.is_contiguous(),
              name, " must be channels_last (4-D) or contiguous (2-D)");
  TORCH_CHECK(t.scalar_type() == kH16 || t.scalar_type() == at::kFloat, name,
              " must be bf16 or fp32");
  check_aligned16(t.data_ptr(), name);
}

int64_t channels_of(const Tensor& x) { return x.size(1); }

std::tuple<Tensor, Tensor, Tensor, Tensor> bn_fwd(Tensor x, c10::optional<Tensor> res,
                                          c10::optional<Tensor> weight,
                                          c10::optional<Tensor> bias, c10::optional<Tensor> rmean,
                                          c10::optional<Tensor> rvar, bool training,
                                          double momentum, double eps, bool relu) {
  const c10::DeviceGuard guard(x.device());
  check_nhwc(x, "x");
  const int64_t C = channels_of(x);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= kMaxBnC, "fused BN needs C % 8 == 0 and C <= ", kMaxBnC, ", got ", C);
  if (res.has_value() && res->defined()) {
    check_nhwc(*res, "res");
    TORCH_CHECK(res->sizes() == x.sizes() && res->scalar_type() == x.scalar_type(),
                "residual must match x");
  }
  auto f32 = x.options().dtype(at::kFloat);
  Tensor y = at::empty_like(x);
  Tensor mean = at::empty({C}, f32), invstd = at::empty({C}, f32);
  Tensor scale_shift = at::empty({2 * C}, f32);
  Tensor scale = scale_shift.narrow(0, 0, C), shift = scale_shift.narrow(0, C, C);
  lw::BNArgs a{};
  a.x = x.data_ptr();
  a.res = (res.has_value() && res->defined()) ? res->data_ptr() : nullptr;
  a.y = y.data_ptr();
  a.M = M;
  a.C = (int)C;
  a.bf16 = x.scalar_type() == kH16;
  a.training = training;
  a.relu = relu;
  a.eps = (float)eps;
  a.momentum = (float)momentum;
  a.gamma = optr<float>(weight);
  a.beta = optr<float>(bias);
  Tensor partial;
  if (training) {
    a.rmean = optr<float>(rmean);
    a.rvar = optr<float>(rvar);
    partial = at::empty({(int64_t)lw::bn_reduce_blocks(M, (int)C) * 2 * C}, f32);
    a.partial = ptr<float>(partial);
    a.mean = ptr<float>(mean);
    a.invstd = ptr<float>(invstd);
    a.scale = ptr<float>(scale);
    a.shift = ptr<float>(shift);
  } else {
    TORCH_CHECK(rmean.has_value() && rvar.has_value(), "eval mode needs running stats");
    mean.copy_(*rmean);
    invstd.copy_(at::rsqrt(*rvar + eps));
    Tensor g = (weight.has_value() && weight->defined()) ? *weight : at::ones({C}, f32);
    Tensor b = (bias.has_value() && bias->defined()) ? *bias : at::zeros({C}, f32);
    scale.copy_(g * invstd);
    shift.copy_(b - mean * scale);
    a.scale = ptr<float>(scale);
    a.shift = ptr<float>(shift);
  }
  lw::bn_forward(a, cur_stream());
  launched("bn_forward");
  // scale/shift as used by the forward: lets the backward recompute the ReLU mask from x
  return {y, mean, invstd, scale_shift};
}

// dgamma/dbeta outputs: fresh tensors, or (dgamma_out/dbeta_out) accumulated into given fp32 [C]
// views — the gradient arena — so no separate add kernel is needed.
static Tensor dparam_out(const c10::optional<Tensor>& t, int64_t C, const Tensor& like,
                         bool& accum) {
  if (t.has_value() && t->defined()) {
    check_dtype(*t, at::kFloat, "dparam_out");
    TORCH_CHECK(t->numel() == C && t->is_contiguous(), "dparam_out must be a contiguous [C]");
    accum = true;
    return *t;
  }
  return at::empty({C}, like.options().dtype(at::kFloat));
}

std::tuple<Tensor, Tensor, Tensor, Tensor> bn_bwd(Tensor dy, Tensor x, c10::optional<Tensor> y,
                                                  c10::optional<Tensor> weight, Tensor mean,
                                                  Tensor invstd, c10::optional<Tensor> scale_shift,
                                                  bool training, bool relu, bool need_dres,
                                                  c10::optional<Tensor> bits,
                                                  c10::optional<Tensor> dgamma_out,
                                                  c10::optional<Tensor> dbeta_out,
                                                  c10::optional<Tensor> stats_rows) {
  const c10::DeviceGuard guard(x.device());
  check_nhwc(x, "x");
  check_nhwc(dy, "dy");
  TORCH_CHECK(dy.scalar_type() == x.scalar_type() && dy.sizes() == x.sizes(), "dy must match x");
  const bool have_ss = scale_shift.has_value() && scale_shift->defined();
  const bool have_bits = bits.has_value() && bits->defined();
  if (have_bits) {
    TORCH_CHECK(bits->scalar_type() == at::kByte && bits->numel() * 8 == x.numel() &&
                bits->is_contiguous(), "bits must be a contiguous uint8 [numel/8] bitmap");
  } else if (relu && !have_ss) {
    TORCH_CHECK(y.has_value() && y->defined(), "relu backward needs the saved output");
    check_nhwc(*y, "y");
  }
  const int64_t C = channels_of(x);
  const int64_t M = x.numel() / C;
  auto f32 = x.options().dtype(at::kFloat);
  Tensor dx = at::empty_like(x);
  Tensor dres = need_dres ? at::empty_like(x) : at::empty({0}, x.options());
  bool accum = false;
  Tensor dgamma = dparam_out(dgamma_out, C, x, accum), dbeta = dparam_out(dbeta_out, C, x, accum);
  Tensor coef = at::empty({3 * C}, f32);
  const bool have_rows = stats_rows.has_value() && stats_rows->defined();
  int64_t nb = lw::bn_reduce_blocks(M, (int)C);
  if (have_rows) {
    // (Σdy', Σdy'·(x−mean)) per M-tile from the producing GEMM's EPI_BSTATS epilogue
    check_dtype(*stats_rows, at::kFloat, "stats_rows");
    TORCH_CHECK(stats_rows->is_cuda() && stats_rows->dim() == 3 && stats_rows->size(1) == 2 &&
                stats_rows->size(2) == C && stats_rows->is_contiguous(),
                "stats_rows must be a contiguous [rows, 2, C] fp32 tensor");
    nb = std::max<int64_t>(nb, lw::colsum_blocks(stats_rows->size(0)));
  }
  Tensor partial = at::empty({nb * 2 * C}, f32);
  lw::BNArgs a{};
  a.accum_dparams = accum;
  if (have_rows) {
    a.stat_rows = ptr<float>(*stats_rows);
    a.stats_rows_n = stats_rows->size(0);
  }
  TORCH_CHECK(!accum || ((dgamma_out.has_value() && dgamma_out->defined()) &&
                         (dbeta_out.has_value() && dbeta_out->defined())),
              "give both dgamma_out and dbeta_out");
  a.x = x.data_ptr();
  a.dy = dy.data_ptr();
  a.bits = (relu && have_bits) ? ptr<uint8_t>(*bits) : nullptr;
  a.y = (relu && !have_ss && !have_bits) ? y->data_ptr() : nullptr;
  if (relu && have_ss && !have_bits) {
    TORCH_CHECK(scale_shift->numel() == 2 * C, "scale_shift must hold 2*C floats");
    a.scale = ptr<float>(*scale_shift);
    a.shift = a.scale + C;
  }
  a.dx = dx.data_ptr();
  a.dres = need_dres ? dres.data_ptr() : nullptr;
  a.M = M;
  a.C = (int)C;
  a.bf16 = x.scalar_type() == kH16;
  a.training = training;
  a.relu = relu;
  a.gamma = optr<float>(weight);
  a.mean = ptr<float>(mean);
  a.invstd = ptr<float>(invstd);
  a.partial = ptr<float>(partial);
  a.dgamma = ptr<float>(dgamma);
  a.dbeta = ptr<float>(dbeta);
  a.A = ptr<float>(coef);
  a.B = a.A + C;
  a.Cc = a.A + 2 * C;
  lw::bn_backward(a, cur_stream());
  launched("bn_backward");
  return {dx, dgamma, dbeta, dres};
}

// Two BN+ReLU backwards that share dy and the forward's ReLU bitmap — a bottleneck's BN3 and its
// downsample BN, both feeding out = relu(bn3(c3) + bnd(cd)): one reduce pass and one apply pass
// read dy and the bitmap once for both (bf16, training). Returns (dx, dx2, dgamma, dbeta,
// dgamma2, dbeta2); the *_out tensors, when given, are accumulated into (arena views).
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> bn_bwd_dual(
    Tensor dy, Tensor x, Tensor x2, Tensor bits, c10::optional<Tensor> weight, Tensor mean,
    Tensor invstd, c10::optional<Tensor> weight2, Tensor mean2, Tensor invstd2,
    c10::optional<Tensor> dgamma_out, c10::optional<Tensor> dbeta_out,
    c10::optional<Tensor> dgamma2_out, c10::optional<Tensor> dbeta2_out) {
  const c10::DeviceGuard guard(x.device());
  check_nhwc(x, "x");
  check_nhwc(x2, "x2");
  check_nhwc(dy, "dy");
  check_dtype(x, kH16, "x");
  TORCH_CHECK(dy.scalar_type() == x.scalar_type() && dy.sizes() == x.sizes() &&
              x2.scalar_type() == x.scalar_type() && x2.sizes() == x.sizes(),
              "dy, x and x2 must match");
  TORCH_CHECK(bits.scalar_type() == at::kByte && bits.numel() * 8 == x.numel() &&
              bits.is_contiguous(), "bits must be a contiguous uint8 [numel/8] bitmap");
  const int64_t C = channels_of(x);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(mean.numel() == C && invstd.numel() == C && mean2.numel() == C &&
              invstd2.numel() == C, "per-channel statistics must hold C floats");
  auto f32 = x.options().dtype(at::kFloat);
  Tensor dx = at::empty_like(x), dx2 = at::empty_like(x);
  bool acc1 = false, acc1b = false, acc2 = false, acc2b = false;
  Tensor dg = dparam_out(dgamma_out, C, x, acc1), db = dparam_out(dbeta_out, C, x, acc1b);
  Tensor dg2 = dparam_out(dgamma2_out, C, x, acc2), db2 = dparam_out(dbeta2_out, C, x, acc2b);
  TORCH_CHECK(acc1 == acc1b && acc2 == acc2b, "give both dgamma_out and dbeta_out of a BN");
  const int64_t nb = lw::bn_reduce_blocks(M, (int)C);
  Tensor partial = at::empty({2 * nb * 2 * C}, f32);
  Tensor coef = at::empty({6 * C}, f32);
  lw::BNArgs a{}, b{};
  for (lw::BNArgs* p : {&a, &b}) {
    p->M = M;
    p->C = (int)C;
    p->bf16 = true;
    p->training = true;
    p->relu = true;
  }
  a.x = x.data_ptr();
  a.dy = dy.data_ptr();
  a.bits = ptr<uint8_t>(bits);
  a.dx = dx.data_ptr();
  a.gamma = optr<float>(weight);
  a.mean = ptr<float>(mean);
  a.invstd = ptr<float>(invstd);
  a.partial = ptr<float>(partial);
  a.dgamma = ptr<float>(dg);
  a.dbeta = ptr<float>(db);
  a.accum_dparams = acc1;
  a.A = ptr<float>(coef);
  a.B = a.A + C;
  a.Cc = a.A + 2 * C;
  b.x = x2.data_ptr();
  b.dx = dx2.data_ptr();
  b.gamma = optr<float>(weight2);
  b.mean = ptr<float>(mean2);
  b.invstd = ptr<float>(invstd2);
  b.partial = a.partial + nb * 2 * C;
  b.dgamma = ptr<float>(dg2);
  b.dbeta = ptr<float>(db2);
  b.accum_dparams = acc2;
  b.A = a.A + 3 * C;
  b.B = a.A + 4 * C;
  b.Cc = a.A + 5 * C;
  lw::bn_backward_dual(a, b, cur_stream());
  launched("bn_backward_dual");
  return {dx, dx2, dg, db, dg2, db2};
}

// ---------------------------------------------------------------- MFMA GEMM
// EPI_BSTATS operands (see lw_kernels.h GemmArgs): the BN input x laid out like the output rows
// ([out_rows][N], ldc == N), its batch mean, and the ReLU mask source — the BN output's bitmap or
// the BN's scale/shift (mask = x*scale+shift > 0).
// The backward-statistics epilogue (gemm_core.h EPI_BSTATS: a data-gradient GEMM also reducing
// the BatchNorm backward it feeds) lost 3.3 % of the ResNet-50 step twice
// (profiles/r2_bstats_ab.log, profiles/r3s2/bstats_cross_ab.txt) and is no longer instantiated:
// the bst_* arguments must be left unset.
static void set_bstats(lw::GemmArgs& g, const c10::optional<Tensor>& bx,
                       const c10::optional<Tensor>& bmean, const c10::optional<Tensor>& bss,
                       const c10::optional<Tensor>& bbits, int64_t out_rows, int64_t N,
                       int64_t ldc, bool out_bf16) {
  (void)g; (void)bmean; (void)bss; (void)bbits; (void)out_rows; (void)N; (void)ldc; (void)out_bf16;
  TORCH_CHECK(!(bx.has_value() && bx->defined()),
              "the backward-statistics GEMM epilogue was removed in round 6 (it lost 3.3 %)");
}

// fp32 slab sets whose split-K reduce was deferred (gemm.hip splitk_flush): held until the flush
// has queued the reduce that reads them
std::vector<Tensor>& splitk_keep() {
  static std::vector<Tensor> keep;
  return keep;
}

int64_t splitk_discard(Tensor dev) {
  const c10::DeviceGuard guard(dev.device());
  const int n = lw::splitk_discard();
  splitk_keep().clear();
  return n;
}

int64_t splitk_pending() { return lw::splitk_pending(); }

// splitk_defer(dev, on): while on, this device's fp32 split-K outputs without bias / ReLU /
// addend (weight gradients accumulated into the gradient arena, ops/block.py) are reduced at
// the next splitk_flush instead of right away. `dev`: any tensor on the device (dispatch).
void splitk_defer(Tensor dev, bool on) {
  const c10::DeviceGuard guard(dev.device());
  lw::splitk_set_defer(on);
}

int64_t splitk_flush(Tensor dev) {
  const c10::DeviceGuard guard(dev.device());
  const int n = lw::splitk_flush(cur_stream());
  // a slab allocated on another stream is read by the reduce just queued on this one: the
  // allocator must not hand its memory out before that reduce has run
  const auto fs = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA();
  for (const Tensor& t : splitk_keep())
    c10::hip::HIPCachingAllocatorMasqueradingAsCUDA::recordStreamMasqueradingAsCUDA(
        t.storage().data_ptr(), fs);
  splitk_keep().clear();
  if (n > 0) launched("splitk_flush");
  return n;
}

std::tuple<Tensor, Tensor> gemm_ex(Tensor A, int64_t lda, bool a_kcontig, Tensor B, int64_t ldb,
                                   bool b_kcontig, int64_t M, int64_t N, int64_t K,
                                   c10::optional<Tensor> bias, bool relu, int64_t splits,
                                   bool out_bf16, int64_t tile, c10::optional<Tensor> pro_scale,
                                   c10::optional<Tensor> pro_shift, bool pro_on_a,
                                   bool want_stats, c10::optional<Tensor> out,
                                   c10::optional<Tensor> addend, bool accumulate, int64_t ldc,
                                   c10::optional<Tensor> addend_bits,
                                   c10::optional<Tensor> bst_x, c10::optional<Tensor> bst_mean,
                                   c10::optional<Tensor> bst_scale_shift,
                                   c10::optional<Tensor> bst_bits) {
  const c10::DeviceGuard guard(A.device());
  TORCH_CHECK(A.is_cuda() && B.is_cuda(), "gemm needs GPU tensors");
  check_dtype(A, kH16, "A");
  check_dtype(B, kH16, "B");
  TORCH_CHECK(A.is_contiguous() && B.is_contiguous(), "gemm operands must be contiguous");
  check_aligned16(A.data_ptr(), "A");
  check_aligned16(B.data_ptr(), "B");
  TORCH_CHECK(M > 0 && N > 0 && K > 0, "empty GEMM");
  TORCH_CHECK(lda % 8 == 0 && ldb % 8 == 0, "leading dimensions must be multiples of 8");
  TORCH_CHECK(K % 8 == 0, "K must be a multiple of 8");
  TORCH_CHECK(a_kcontig || M % 8 == 0, "M must be a multiple of 8 for an M-contiguous A");
  TORCH_CHECK(b_kcontig || N % 8 == 0, "N must be a multiple of 8 for an N-contiguous B");
  TORCH_CHECK(A.numel() >= (a_kcontig ? (M - 1) * lda + K : (K - 1) * lda + M), "A too small");
  TORCH_CHECK(B.numel() >= (b_kcontig ? (N - 1) * ldb + K : (K - 1) * ldb + N), "B too small");
  TORCH_CHECK((tile >= 0 && tile <= 6) || (tile >= 11 && tile <= 13) || (tile >= 21 && tile <= 24) ||
                  lw::gemm_is_mf32((int)tile),
              "tile id");
  if (ldc <= 0) ldc = N;
  TORCH_CHECK(ldc >= N, "ldc must be >= N");
  const auto odt = out_bf16 ? kH16 : at::kFloat;
  Tensor C;
  if (out.has_value() && out->defined()) {
    C = *out;
    TORCH_CHECK(C.is_cuda() && C.scalar_type() == odt, "out dtype must match out_bf16");
    TORCH_CHECK(C.is_contiguous(at::MemoryFormat::ChannelsLast) || C.is_contiguous(),
                "out must be dense");
    TORCH_CHECK(C.numel() >= (M - 1) * ldc + N, "out too small for [M, ldc]");
    TORCH_CHECK(out_bf16 ? ldc % 8 == 0 : ldc % 4 == 0, "ldc alignment");
    check_aligned16(C.data_ptr(), "out");
  } else {
    TORCH_CHECK(!accumulate, "accumulate needs an out tensor");
    TORCH_CHECK(ldc == N, "ldc != N needs an out tensor");
    C = at::empty({M, N}, A.options().dtype(odt));
  }
  TORCH_CHECK(!accumulate || !out_bf16, "accumulate is for fp32 outputs");
  TORCH_CHECK(A.numel() * 2 < (1LL << 31) && B.numel() * 2 < (1LL << 31),
              "gemm operands must be < 2 GiB (32-bit buffer offsets)");
  lw::GemmArgs g{};
  g.a_bytes = (uint32_t)(A.numel() * 2);
  g.b_bytes = (uint32_t)(B.numel() * 2);
  g.A = ptr<uint16_t>(A);
  g.lda = lda;
  g.a_kcontig = a_kcontig;
  g.B = ptr<uint16_t>(B);
  g.ldb = ldb;
  g.b_kcontig = b_kcontig;
  g.C = C.data_ptr();
  g.ldc = ldc;
  g.out_bf16 = out_bf16;
  g.accumulate = accumulate;
  if (addend.has_value() && addend->defined()) {
    TORCH_CHECK(out_bf16, "addend needs a bf16 output");
    check_dtype(*addend, kH16, "addend");
    TORCH_CHECK(addend->numel() >= (M - 1) * ldc + N, "addend too small for [M, ldc]");
    TORCH_CHECK(addend->is_contiguous(at::MemoryFormat::ChannelsLast) || addend->is_contiguous(),
                "addend must be dense");
    check_aligned16(addend->data_ptr(), "addend");
    g.addend = ptr<uint16_t>(*addend);
    if (addend_bits.has_value() && addend_bits->defined()) {
      TORCH_CHECK(ldc == N && addend_bits->scalar_type() == at::kByte &&
                  addend_bits->numel() * 8 >= M * N && N % 8 == 0,
                  "addend_bits: uint8 bitmap of the [M, N] addend (ldc == N, N % 8 == 0)");
      g.add_bits = ptr<uint8_t>(*addend_bits);
    }
  }
  if (bias.has_value() && bias->defined()) {
    check_dtype(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() == N && bias->is_contiguous(), "bias size");
    g.bias = ptr<float>(*bias);
  }
  g.relu = relu;
  g.M = (int)M;
  g.N = (int)N;
  g.K = (int)K;
  g.splits = (int)splits;
  g.tile = (int)tile;
  const bool pro = pro_scale.has_value() && pro_scale->defined();
  if (pro) {
    TORCH_CHECK(pro_shift.has_value() && pro_shift->defined(), "prologue needs scale and shift");
    const int64_t n = pro_on_a ? K : N;
    TORCH_CHECK(pro_on_a ? a_kcontig : !b_kcontig,
                "prologue: per-k on a K-contiguous A or per-n on an N-contiguous B");
    for (const Tensor* t : {&*pro_scale, &*pro_shift}) {
      check_dtype(*t, at::kFloat, "prologue");
      TORCH_CHECK(t->numel() >= n && t->is_contiguous(), "prologue vector size");
      check_aligned16(t->data_ptr(), "prologue");
    }
    g.pro_scale = ptr<float>(*pro_scale);
    g.pro_shift = ptr<float>(*pro_shift);
    g.pro_on_a = pro_on_a;
  }
  if (tile >= 11 && tile <= 13)
    TORCH_CHECK(lw::gemm_stream_ok(g), "streaming GEMM tile ", tile, " does not support this "
                "problem (needs K-contiguous A, K in {64,128,256}, bf16 out, no split-K)");
  const int zs = lw::gemm_splits_used(g);
  Tensor partial, stats;
  if (zs > 1) {
    partial = at::empty({(int64_t)zs * M * N}, A.options().dtype(at::kFloat));
    g.partial = ptr<float>(partial);
  }
  set_bstats(g, bst_x, bst_mean, bst_scale_shift, bst_bits, M, N, ldc, out_bf16);
  if (g.bst_x) {
    TORCH_CHECK(want_stats && a_kcontig && !b_kcontig && !pro && (tile < 11 || lw::gemm_is_mf32((int)tile)),
                "backward statistics: a tiled data-gradient GEMM (K-contiguous A, N-contiguous "
                "B, no prologue) with want_stats");
  }
  if (want_stats) {
    TORCH_CHECK(zs == 1, "column statistics need splits == 1");
    stats = at::empty({(int64_t)lw::gemm_tiles_m(g), 2, N}, A.options().dtype(at::kFloat));
    g.stats = ptr<float>(stats);
  } else {
    stats = at::empty({0}, A.options().dtype(at::kFloat));
  }
  lw::gemm_bf16(g, cur_stream());
  if (zs > 1 && lw::splitk_take_deferred()) splitk_keep().push_back(partial);
  launched("gemm_bf16");
  return {C, stats};
}

Tensor gemm(Tensor A, int64_t lda, bool a_kcontig, Tensor B, int64_t ldb, bool b_kcontig,
            int64_t M, int64_t N, int64_t K, c10::optional<Tensor> bias, bool relu,
            int64_t splits, bool out_bf16) {
  return std::get<0>(gemm_ex(A, lda, a_kcontig, B, ldb, b_kcontig, M, N, K, bias, relu, splits,
                             out_bf16, 0, c10::nullopt, c10::nullopt, true, false, c10::nullopt,
                             c10::nullopt, false, 0, c10::nullopt, c10::nullopt, c10::nullopt,
                             c10::nullopt, c10::nullopt));
}

// ---------------------------------------------------------------- implicit-GEMM convolution
// G: the gathered NHWC bf16 tensor; Op: the other GEMM operand — the packed weights (row-gather
// modes 1/2: [N][K] for the forward, b_kcontig, or per-class [K_c][N] slabs for the data
// gradient) or dY [pixels][M] (weight-gradient modes 3/4). geom = [Nb, Hin, Win, C, sh, sw, dh,
// dw, Hout, Wout, osy, osx, nclass, then per class TR, TS, oh, ow, Hg, Wg, py, px, K, b_off].
// Every index the kernels can form is checked here against the tensors' sizes.
// K-contiguous data-gradient weight pack (csrc/conv.hip k_pack_dgrad_kc): w is a bf16
// channels_last [Co, C, R, S] weight; cls = 4 ints (r0, s0, TR, TS) per parity class.
// pack_dgrad_kc of several weights in one launch: w[i] (channels_last [Co][C][R][S] memory, or a
// contiguous [Co][C] for a 1x1) into out[i] ([nclass][C][kmax]); prm: 20 ints per job —
// [sh, sw, kmax, nclass, r0 x4, s0 x4, TR x4, TS x4] as pack_dgrad_kc's arguments (padded to 4
// classes); kmax = 0 packs pack_dgrad_nkc's [K][C] slabs instead
void pack_kc_multi(std::vector<Tensor> w, std::vector<Tensor> out, std::vector<int64_t> prm) {
  TORCH_CHECK(w.size() == out.size() && prm.size() == 20 * w.size(), "pack_kc_multi: list sizes");
  if (w.empty()) return;
  const c10::DeviceGuard guard(w[0].device());
  std::vector<const uint16_t*> wp;
  std::vector<uint16_t*> op;
  std::vector<int> p;
  for (size_t i = 0; i < w.size(); ++i) {
    check_dtype(w[i], kH16, "weight");
    check_dtype(out[i], kH16, "out");
    const bool cl = w[i].dim() == 4 && (w[i].is_contiguous(at::MemoryFormat::ChannelsLast) ||
                                        (w[i].size(2) == 1 && w[i].size(3) == 1 &&
                                         w[i].is_contiguous()));
    TORCH_CHECK(w[i].is_cuda() && cl && out[i].is_contiguous() && w[i].device() == w[0].device()
                && out[i].device() == w[0].device(),
                "pack_kc_multi: channels_last 4-d GPU weights on one device");
    const int64_t* q = prm.data() + 20 * i;
    const int Co = (int)w[i].size(0), C = (int)w[i].size(1), R = (int)w[i].size(2),
              S = (int)w[i].size(3);
    const int sh = (int)q[0], sw = (int)q[1], kmax = (int)q[2], nclass = (int)q[3];
    // kmax == 0: the [K][C] form (pack_dgrad_nkc: positive strides, C % 8, 16-byte loads)
    const bool nkc = kmax == 0;
    TORCH_CHECK(nclass >= 1 && nclass <= 4 && kmax >= 0 && kmax % 8 == 0 &&
                (sh >= 1 || (sh == -1 && !nkc)) && (sw >= 1 || (sw == -1 && !nkc)) &&
                (!nkc || C % 8 == 0), "pack_kc_multi: classes / kmax / strides");
    int64_t total = 0;
    for (int k = 0; k < nclass; ++k) {
      const int64_t r0 = q[4 + k], s0 = q[8 + k], TR = q[12 + k], TS = q[16 + k];
      const int64_t rl = r0 + sh * (TR - 1), sl = s0 + sw * (TS - 1);
      TORCH_CHECK(r0 >= 0 && s0 >= 0 && TR >= 1 && TS >= 1 && r0 < R && s0 < S && rl >= 0 &&
                  rl < R && sl >= 0 && sl < S && (nkc || TR * TS * Co <= kmax),
                  "pack_kc_multi: class taps outside the kernel window");
      total += nkc ? TR * TS * Co * C : (int64_t)C * kmax;
    }
    TORCH_CHECK(out[i].numel() == total, "pack_kc_multi: out size");
    if (nkc) check_aligned16(w[i].data_ptr(), "weight");
    check_aligned16(out[i].data_ptr(), "out");
    wp.push_back(ptr<uint16_t>(w[i]));
    op.push_back(ptr<uint16_t>(out[i]));
    const int row[8] = {Co, C, R, S, sh, sw, nclass, kmax};
    for (int k = 0; k < 8; ++k) p.push_back(row[k]);
    for (int k = 0; k < 16; ++k) p.push_back((int)q[4 + k]);
  }
  lw::pack_kc_multi(wp.data(), op.data(), p.data(), (int)w.size(), cur_stream());
  launched("pack_kc_multi");
}

Tensor pack_dgrad_kc(Tensor w, std::vector<int64_t> cls, int64_t sh, int64_t sw, int64_t kmax) {
  const c10::DeviceGuard guard(w.device());
  TORCH_CHECK(w.is_cuda() && w.dim() == 4, "pack_dgrad_kc: a 4-d GPU weight");
  check_dtype(w, kH16, "weight");
  TORCH_CHECK(w.is_contiguous(at::MemoryFormat::ChannelsLast) || (w.size(2) == 1 && w.size(3) == 1
              && w.is_contiguous()), "weight must be channels_last [Co][R][S][C] in memory");
  const int Co = (int)w.size(0), C = (int)w.size(1), R = (int)w.size(2), S = (int)w.size(3);
  const int nclass = (int)(cls.size() / 4);
  TORCH_CHECK(cls.size() % 4 == 0 && nclass >= 1 && nclass <= 4, "cls: 1..4 classes of 4 ints");
  // sh / sw = -1 walks the window backwards: the flipped weight of a 3x3/1 data gradient run as
  // a forward conv (ops/conv.py tap_dgrad_weight: r0 = s0 = 2, stride -1)
  TORCH_CHECK(kmax % 8 == 0 && (sh >= 1 || sh == -1) && (sw >= 1 || sw == -1), "kmax / strides");
  int r0[4], s0[4], TR[4], TS[4];
  for (int i = 0; i < nclass; ++i) {
    r0[i] = (int)cls[4 * i]; s0[i] = (int)cls[4 * i + 1];
    TR[i] = (int)cls[4 * i + 2]; TS[i] = (int)cls[4 * i + 3];
    const int64_t rl = r0[i] + sh * (TR[i] - 1), sl = s0[i] + sw * (TS[i] - 1);
    TORCH_CHECK(r0[i] >= 0 && s0[i] >= 0 && TR[i] >= 1 && TS[i] >= 1 && r0[i] < R &&
                s0[i] < S && rl >= 0 && rl < R && sl >= 0 && sl < S &&
                (int64_t)TR[i] * TS[i] * Co <= kmax, "class taps outside the kernel window");
  }
  Tensor out = at::empty({(int64_t)nclass * C * kmax}, w.options());
  lw::pack_dgrad_kc(ptr<uint16_t>(w), ptr<uint16_t>(out), Co, C, R, S, (int)sh, (int)sw, nclass,
                    r0, s0, TR, TS, (int)kmax, cur_stream());
  launched("pack_dgrad_kc");
  return out;
}

// [K][C] per-class slabs Wt_c[jr][js][co][ci] = w[co, ci, r0 + sh*jr, s0 + sw*js], concatenated
// (ops/conv.py pack_dgrad_weight): w channels_last bf16/fp16 [Co][C][R][S], C % 8 == 0
Tensor pack_dgrad_nkc(Tensor w, std::vector<int64_t> cls, int64_t sh, int64_t sw) {
  const c10::DeviceGuard guard(w.device());
  TORCH_CHECK(w.is_cuda() && w.dim() == 4 && w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "pack_dgrad_nkc: a channels_last 4-d GPU weight");
  check_dtype(w, kH16, "weight");
  check_aligned16(w.data_ptr(), "weight");
  const int Co = (int)w.size(0), C = (int)w.size(1), R = (int)w.size(2), S = (int)w.size(3);
  TORCH_CHECK(C % 8 == 0, "pack_dgrad_nkc: C % 8 == 0");
  const int nclass = (int)(cls.size() / 4);
  TORCH_CHECK(cls.size() % 4 == 0 && nclass >= 1 && nclass <= 4 && sh >= 1 && sw >= 1,
              "cls: 1..4 classes of 4 ints; positive strides");
  int r0[4], s0[4], TR[4], TS[4];
  int64_t total = 0;
  for (int i = 0; i < nclass; ++i) {
    r0[i] = (int)cls[4 * i]; s0[i] = (int)cls[4 * i + 1];
    TR[i] = (int)cls[4 * i + 2]; TS[i] = (int)cls[4 * i + 3];
    TORCH_CHECK(r0[i] >= 0 && s0[i] >= 0 && TR[i] >= 1 && TS[i] >= 1 &&
                r0[i] + sh * (TR[i] - 1) < R && s0[i] + sw * (TS[i] - 1) < S,
                "class taps outside the kernel window");
    total += (int64_t)TR[i] * TS[i] * Co * C;
  }
  Tensor out = at::empty({total}, w.options());
  lw::pack_dgrad_nkc(ptr<uint16_t>(w), ptr<uint16_t>(out), Co, C, R, S, (int)sh, (int)sw, nclass,
                     r0, s0, TR, TS, cur_stream());
  launched("pack_dgrad_nkc");
  return out;
}

std::tuple<Tensor, Tensor> conv_ex(Tensor G, Tensor Op, int64_t mode, std::vector<int64_t> geom,
                                   int64_t N, int64_t tile, int64_t splits, bool out_bf16,
                                   c10::optional<Tensor> pro_scale, c10::optional<Tensor> pro_shift,
                                   bool want_stats, c10::optional<Tensor> out, bool accumulate,
                                   int64_t ldc, bool b_kcontig, int64_t ldb,
                                   c10::optional<Tensor> addend, c10::optional<Tensor> bst_x,
                                   c10::optional<Tensor> bst_mean,
                                   c10::optional<Tensor> bst_scale_shift,
                                   c10::optional<Tensor> bst_bits, c10::optional<Tensor> bias,
                                   bool relu) {
  const c10::DeviceGuard guard(G.device());
  TORCH_CHECK(G.is_cuda() && Op.is_cuda(), "conv needs GPU tensors");
  check_dtype(G, kH16, "gathered tensor");
  check_dtype(Op, kH16, "operand");
  TORCH_CHECK(G.is_contiguous() || G.is_contiguous(at::MemoryFormat::ChannelsLast),
              "gathered tensor must be dense NHWC");
  TORCH_CHECK(Op.is_contiguous() || Op.is_contiguous(at::MemoryFormat::ChannelsLast),
              "operand must be dense (dY channels_last)");
  TORCH_CHECK(mode >= lw::CV_A && mode <= lw::CV_B4, "conv mode");
  TORCH_CHECK(lw::conv_tile_ok((int)mode, (int)tile), "tile ", tile, " not built for conv mode ",
              mode);
  TORCH_CHECK(geom.size() >= 13, "geom too short");
  const int64_t Nb = geom[0];
  lw::ConvGeomHost h{};
  h.Hin = (int)geom[1]; h.Win = (int)geom[2]; h.C = (int)geom[3];
  h.sh = (int)geom[4]; h.sw = (int)geom[5]; h.dh = (int)geom[6]; h.dw = (int)geom[7];
  h.Hout = (int)geom[8]; h.Wout = (int)geom[9]; h.osy = (int)geom[10]; h.osx = (int)geom[11];
  h.nclass = (int)geom[12];
  TORCH_CHECK(h.nclass >= 1 && h.nclass <= 4 && geom.size() == 13 + 10 * (size_t)h.nclass,
              "geom: 1..4 classes of 10 ints");
  TORCH_CHECK(std::abs(h.dh) == 1 && std::abs(h.dw) == 1 && h.sh >= 1 && h.sw >= 1 &&
              h.osy >= 1 && h.osx >= 1, "geom: strides / directions");
  const bool ga = mode == lw::CV_A || mode == lw::CV_A4;
  const bool c4 = mode == lw::CV_A4 || mode == lw::CV_B4;
  TORCH_CHECK(c4 ? h.C == 4 : (h.C > 0 && h.C % 8 == 0),
              c4 ? "4-channel mode needs C == 4" : "conv needs C % 8 == 0");
  TORCH_CHECK(G.numel() >= Nb * h.Hin * h.Win * h.C, "gathered tensor smaller than geom");
  TORCH_CHECK(Nb * h.Hin * h.Win < (1LL << 31), "gathered tensor too large");
  check_aligned16(G.data_ptr(), "gathered tensor");
  check_aligned16(Op.data_ptr(), "operand");
  int64_t Mmax = 0;
  for (int i = 0; i < h.nclass; ++i) {
    const int64_t* c = &geom[13 + 10 * i];
    h.TR[i] = (int)c[0]; h.TS[i] = (int)c[1]; h.oh[i] = (int)c[2]; h.ow[i] = (int)c[3];
    h.Hg[i] = (int)c[4]; h.Wg[i] = (int)c[5]; h.py[i] = (int)c[6]; h.px[i] = (int)c[7];
    h.K[i] = (int)c[8]; h.b_off[i] = c[9];
    TORCH_CHECK(h.TR[i] >= 0 && h.TS[i] >= 1 && h.Hg[i] >= 1 && h.Wg[i] >= 1, "class geometry");
    TORCH_CHECK(!c4 || h.TS[i] % 2 == 0, "4-channel mode needs an even tap count along w");
    TORCH_CHECK((int64_t)h.K[i] == (int64_t)h.TR[i] * h.TS[i] * h.C || (!ga),
                "class K must be taps * C");
    const int64_t Mc = Nb * h.Hg[i] * h.Wg[i];
    TORCH_CHECK(Mc < (1LL << 24), "pixel count beyond the fp32 fast divide");
    h.M[i] = (int)Mc;
    Mmax = std::max(Mmax, Mc);
    if (h.osy > 1 || h.osx > 1 || h.nclass > 1) {
      TORCH_CHECK((int64_t)(h.Hg[i] - 1) * h.osy + h.py[i] < h.Hout &&
                  (int64_t)(h.Wg[i] - 1) * h.osx + h.px[i] < h.Wout && h.py[i] >= 0 &&
                  h.px[i] >= 0, "class output map outside the output grid");
    }
  }
  TORCH_CHECK(N > 0 && N % 8 == 0, "conv GEMM N must be a positive multiple of 8");
  TORCH_CHECK(G.numel() * 2 < (1LL << 31) && Op.numel() * 2 < (1LL << 31),
              "conv operands must be < 2 GiB (32-bit buffer offsets)");
  lw::GemmArgs g{};
  g.tile = (int)tile;
  g.out_bf16 = out_bf16;
  g.accumulate = accumulate;
  g.N = (int)N;
  Tensor C;
  if (ga) {
    TORCH_CHECK(out_bf16 && !accumulate, "row-gather convs write bf16");
    for (int i = 0; i < h.nclass; ++i) {
      const int64_t need = b_kcontig ? h.b_off[i] + (N - 1) * ldb + h.K[i]
                                     : h.b_off[i] + (int64_t)(h.K[i] - 1) * ldb + N;
      TORCH_CHECK(h.K[i] == 0 || Op.numel() >= need, "weight operand too small for class ", i);
      TORCH_CHECK(h.b_off[i] % 8 == 0, "class weight offset alignment");
    }
    TORCH_CHECK(ldb % 8 == 0 && ldb >= (b_kcontig ? *std::max_element(h.K, h.K + h.nclass) : N),
                "ldb");
    g.M = (int)Mmax;
    g.K = *std::max_element(h.K, h.K + h.nclass);   // one K range per workgroup: the largest
    g.A = ptr<uint16_t>(G);
    g.a_bytes = (uint32_t)(G.numel() * 2);
    g.b_bytes = (uint32_t)(Op.numel() * 2);
    g.lda = h.C;
    g.a_kcontig = true;
    g.B = ptr<uint16_t>(Op);
    g.ldb = ldb;
    g.b_kcontig = b_kcontig;
    g.splits = 1;
    if (h.nclass == 1 && h.osy == 1 && h.osx == 1)
      TORCH_CHECK(h.M[0] <= Nb * h.Hout * h.Wout, "rows beyond the output grid");
  } else {
    TORCH_CHECK(h.nclass == 1, "weight gradients take one class");
    TORCH_CHECK(!out_bf16, "weight gradients are fp32");
    TORCH_CHECK(N == (int64_t)h.TR[0] * h.TS[0] * h.C, "wgrad N must be taps * C");
    g.M = (int)(ldb);                          // ldb carries Co (= M) for the weight gradient
    TORCH_CHECK(g.M > 0 && g.M % 8 == 0, "wgrad: Co must be a multiple of 8");
    g.K = h.M[0];                              // reduction over the output pixels
    TORCH_CHECK(Op.numel() >= (int64_t)g.K * g.M, "dY smaller than pixels x Co");
    g.A = ptr<uint16_t>(Op);
    g.a_bytes = (uint32_t)(Op.numel() * 2);
    g.b_bytes = (uint32_t)(G.numel() * 2);
    g.lda = g.M;
    g.a_kcontig = false;
    g.B = ptr<uint16_t>(G);
    g.ldb = 0;
    g.b_kcontig = false;
    g.splits = (int)std::max<int64_t>(splits, 1);
  }
  if (ldc <= 0) ldc = N;
  TORCH_CHECK(ldc >= N && (out_bf16 ? ldc % 8 == 0 : ldc % 4 == 0), "ldc");
  const int64_t out_rows = ga ? Nb * h.Hout * h.Wout : g.M;
  const auto odt = out_bf16 ? kH16 : at::kFloat;
  if (out.has_value() && out->defined()) {
    C = *out;
    TORCH_CHECK(C.is_cuda() && C.scalar_type() == odt, "out dtype");
    TORCH_CHECK(C.is_contiguous() || C.is_contiguous(at::MemoryFormat::ChannelsLast),
                "out must be dense");
    TORCH_CHECK(C.numel() >= (out_rows - 1) * ldc + N, "out too small");
    check_aligned16(C.data_ptr(), "out");
  } else {
    TORCH_CHECK(!accumulate, "accumulate needs an out tensor");
    C = at::empty({out_rows, ldc}, G.options().dtype(odt));
    if (ga && (h.nclass > 1 || h.osy > 1 || h.osx > 1)) {
      // the parity classes are disjoint pixel sets: zero only when some pixel has no class
      int64_t covered = 0;
      bool disjoint = true;
      for (int i = 0; i < h.nclass; ++i) {
        covered += (int64_t)h.Hg[i] * h.Wg[i];
        disjoint = disjoint && h.py[i] < h.osy && h.px[i] < h.osx;
        for (int j = 0; j < i; ++j) disjoint = disjoint && (h.py[j] != h.py[i] || h.px[j] != h.px[i]);
      }
      if (!disjoint || covered != (int64_t)h.Hout * h.Wout) C.zero_();
    }
  }
  g.C = C.data_ptr();
  g.ldc = ldc;
  if (pro_scale.has_value() && pro_scale->defined()) {
    TORCH_CHECK(ga && b_kcontig && !c4, "BN prologue: forward convs with C % 8 == 0 only");
    TORCH_CHECK(pro_shift.has_value() && pro_shift->defined(), "prologue needs scale and shift");
    for (const Tensor* t : {&*pro_scale, &*pro_shift}) {
      check_dtype(*t, at::kFloat, "prologue");
      TORCH_CHECK(t->numel() >= h.C && t->is_contiguous(), "prologue vector size");
      check_aligned16(t->data_ptr(), "prologue");
    }
    g.pro_scale = ptr<float>(*pro_scale);
    g.pro_shift = ptr<float>(*pro_shift);
    g.pro_on_a = ga;
  }
  if (addend.has_value() && addend->defined()) {
    // bf16 [out_rows][ldc] added after rounding, indexed by output row (may alias `out`)
    TORCH_CHECK(ga && out_bf16 && !accumulate, "conv addend: bf16 row-gather (fwd/dgrad) output");
    check_dtype(*addend, kH16, "addend");
    TORCH_CHECK(addend->is_cuda() && (addend->is_contiguous() ||
                addend->is_contiguous(at::MemoryFormat::ChannelsLast)), "addend must be dense");
    TORCH_CHECK(addend->numel() >= (out_rows - 1) * ldc + N, "addend too small");
    check_aligned16(addend->data_ptr(), "addend");
    g.addend = ptr<uint16_t>(*addend);
  }
  const int zs = ga ? 1 : lw::conv_splits_used(g);
  Tensor partial, stats;
  if (zs > 1) {
    partial = at::empty({(int64_t)zs * g.M * N}, G.options().dtype(at::kFloat));
    g.partial = ptr<float>(partial);
  }
  set_bstats(g, bst_x, bst_mean, bst_scale_shift, bst_bits, out_rows, N, ldc, out_bf16);
  if (want_stats && g.bst_x) {
    // data-gradient conv that also does the reduce pass of the BN its output feeds: one stats
    // row per (parity class, M-tile); rows of tiles a smaller class skips stay zero
    TORCH_CHECK(ga && !b_kcontig && !c4 && g.pro_scale == nullptr && zs == 1,
                "backward statistics: data-gradient convs only");
    int bm, bn, bk;
    lw::gemm_tile_shape(g.tile, bm, bn, bk);
    stats = at::zeros({(int64_t)h.nclass * ((g.M + bm - 1) / bm), 2, N},
                      G.options().dtype(at::kFloat));
    g.stats = ptr<float>(stats);
  } else if (want_stats) {
    TORCH_CHECK(!g.bst_x, "backward statistics need want_stats");
    TORCH_CHECK(ga && b_kcontig && h.nclass == 1, "column statistics: forward convs only");
    const int bm = lw::stats_rows_bm(g.tile);
    stats = at::empty({(g.M + bm - 1) / bm, 2, N}, G.options().dtype(at::kFloat));
    g.stats = ptr<float>(stats);
  } else {
    TORCH_CHECK(!g.bst_x, "backward statistics need want_stats");
    stats = at::empty({0}, G.options().dtype(at::kFloat));
  }
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(ga && out_bf16 && !g.bst_x, "conv bias epilogue: forward convs only");
    check_dtype(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->is_cuda() && bias->numel() >= N && bias->is_contiguous(), "bias [N] fp32");
    g.bias = ptr<float>(*bias);
  }
  TORCH_CHECK(!relu || (ga && out_bf16 && !g.bst_x), "conv ReLU epilogue: forward convs only");
  g.relu = relu;
  if (tile == lw::GEMM_B256 || tile == lw::GEMM_B256x128)
    TORCH_CHECK((mode == lw::CV_A || mode == lw::CV_B) && lw::conv_big_ok(g, h),
                "conv big tiles: one-class row gather, C % 64 == 0, K-contiguous weight, no "
                "prologue / addend / backward statistics");
  lw::conv_gemm(g, h, (int)mode, cur_stream());
  if (zs > 1 && lw::splitk_take_deferred()) splitk_keep().push_back(partial);
  launched("conv_gemm");
  return {C, stats};
}

// Direct stem convolution (conv.hip k_stem_conv7): x4 [N, 4, H, W] bf16 channels_last (the image
// padded to 4 channels), w the packed [64][224] operand of pack_fwd_weight; returns
// (y [N, 64, Ho, Wo] channels_last, stats [workgroups, 2, 64]).
std::tuple<Tensor, Tensor> stem_conv7(Tensor x, Tensor w) {
  const c10::DeviceGuard guard(x.device());
  check_dtype(x, kH16, "x");
  check_dtype(w, kH16, "w");
  TORCH_CHECK(x.is_cuda() && w.is_cuda() && x.dim() == 4 && x.size(1) == 4 &&
              x.is_contiguous(at::MemoryFormat::ChannelsLast), "x: [N, 4, H, W] channels_last");
  TORCH_CHECK(w.is_contiguous() && w.numel() == 64 * 224, "w: packed [64][224]");
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3);
  const int64_t Ho = (H + 6 - 7) / 2 + 1, Wo = (W + 6 - 7) / 2 + 1;
  TORCH_CHECK(lw::stem_conv7_ok(4, 64, 7, 7, 2, 2, 3, 3, (int)H, (int)W, (int)Ho, (int)Wo),
              "stem_conv7: unsupported geometry");
  TORCH_CHECK(N * H * W * 8 < (1LL << 31) && N * Ho * Wo * 128 < (1LL << 40), "stem_conv7 size");
  check_aligned16(x.data_ptr(), "x");
  check_aligned16(w.data_ptr(), "w");
  Tensor y = at::empty({N, 64, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor st = at::empty({lw::stem_conv7_blocks((int)N, (int)Ho), 2, 64}, x.options().dtype(at::kFloat));
  lw::stem_conv7(ptr<uint16_t>(x), ptr<uint16_t>(w), ptr<uint16_t>(y), ptr<float>(st), (int)N,
                 (int)H, (int)W, (int)Ho, (int)Wo, cur_stream());
  launched("stem_conv7");
  return {y, st};
}

// Tap-reuse 3x3 / stride-1 / pad-1 convolution (conv3tap.hip k_conv3_tap): x [N, C, H, W] bf16
// channels_last, w the K-contiguous [Co][9C] operand ((r, s, ci) order; for a data gradient the
// flipped, transposed weight); returns (y [N, Co, H, W] channels_last, stats [tiles_m, 2, Co] or
// an empty tensor).
std::tuple<Tensor, Tensor> conv3_tap(Tensor x, Tensor w, int64_t Co, bool want_stats) {
  const c10::DeviceGuard guard(x.device());
  check_dtype(x, kH16, "x");
  check_dtype(w, kH16, "w");
  TORCH_CHECK(x.is_cuda() && w.is_cuda() && x.dim() == 4 &&
              x.is_contiguous(at::MemoryFormat::ChannelsLast), "x: [N, C, H, W] channels_last");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(w.is_contiguous() && w.numel() == Co * 9 * C, "w: [Co][9C] K-contiguous");
  TORCH_CHECK(lw::conv3_tap_ok((int)C, (int)Co, (int)H, (int)W), "conv3_tap: unsupported geometry");
  TORCH_CHECK(x.numel() * 2 < (1LL << 31) && w.numel() * 2 < (1LL << 31), "conv3_tap: operand > 2 GiB");
  check_aligned16(x.data_ptr(), "x");
  check_aligned16(w.data_ptr(), "w");
  Tensor y = at::empty({N, Co, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int64_t rows = lw::conv3_tap_tiles_m((int)N, (int)H, (int)W);
  Tensor st = want_stats ? at::empty({rows, 2, Co}, x.options().dtype(at::kFloat))
                         : at::empty({0}, x.options().dtype(at::kFloat));
  lw::conv3_tap(ptr<uint16_t>(x), ptr<uint16_t>(w), ptr<uint16_t>(y),
                want_stats ? ptr<float>(st) : nullptr, (int)N, (int)H, (int)W, (int)C, (int)Co,
                cur_stream());
  launched("conv3_tap");
  return {y, st};
}

// A bottleneck's BN3 backward (bf16, training, ReLU bitmap) with its apply fused into the two
// GEMMs that consume dc3 (bnfuse.hip k_bn3_bwd_dgemm): reduce + finalize as bn_bwd, then one
// kernel forms dc3 tile by tile and writes da2 = dc3·W3 ([M, Ci] bf16) and dW3 = dc3ᵀ·a2 as fp32
// slabs ((C, Ci) = (256, 64) or (512, 128): the ResNet-50 stage-1 / stage-2 BN3), summed into dw_out (accumulated: the gradient arena view [C][Ci]) or a fresh [C, Ci]
// by the fixed-order split-K reduce (deferred inside a splitk_defer scope). w3t is W3ᵀ [Ci][C].
// With x2 (a downsample block: the shortcut BN's input, fed by the same dy and bitmap) the dual
// reduce runs and the same pass also writes that BN's dx2 (as bn_bwd_dual's). Returns (da2, dW3,
// dgamma, dbeta, dx2, dgamma2, dbeta2) (the last three empty without x2); dc3 is never written.
// With bn2_x (c2 [M][Ci], BN2's input), bn2_ss (its forward scale | shift) and bn2_mean, the
// kernel also reduces BN2's backward sums from the da2 tiles it writes; the 8th output holds
// them as [slabs, 2, Ci] rows for bn_bwd(..., stats_rows=) (empty otherwise). With
// a2_from_bn2, `a2` is c2 (BN2's input) and the kernel forms a2 = relu(bn2(c2)) from bn2_ss itself.
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> bn3_bwd_fused(
    Tensor dy, Tensor x, Tensor bits, c10::optional<Tensor> weight, Tensor mean, Tensor invstd,
    Tensor w3t, Tensor a2, c10::optional<Tensor> dw_out, c10::optional<Tensor> dgamma_out,
    c10::optional<Tensor> dbeta_out, c10::optional<Tensor> x2, c10::optional<Tensor> weight2,
    c10::optional<Tensor> mean2, c10::optional<Tensor> invstd2,
    c10::optional<Tensor> dgamma2_out, c10::optional<Tensor> dbeta2_out,
    c10::optional<Tensor> bn2_x, c10::optional<Tensor> bn2_ss, c10::optional<Tensor> bn2_mean,
    bool a2_from_bn2) {
  const c10::DeviceGuard guard(x.device());
  const bool dual = x2.has_value() && x2->defined();
  const bool s2 = bn2_x.has_value() && bn2_x->defined();
  for (const Tensor* t : {&dy, &x, &w3t, &a2}) {
    check_dtype(*t, kH16, "bn3_bwd_fused operand");
    TORCH_CHECK(t->is_cuda() && t->dim() == 2 && t->is_contiguous(),
                "bn3_bwd_fused: contiguous 2-D [rows, channels] operands");
    check_aligned16(t->data_ptr(), "bn3_bwd_fused operand");
  }
  const int64_t M = x.size(0), C = x.size(1), Ci = a2.size(1);
  TORCH_CHECK(dy.sizes() == x.sizes() && a2.size(0) == M, "dy / a2 rows must match x");
  TORCH_CHECK(w3t.size(0) == Ci && w3t.size(1) == C, "w3t must be W3ᵀ [Ci][C]");
  TORCH_CHECK(lw::bn3_bwd_dgemm_ok(M, (int)C, (int)Ci),
              "bn3_bwd_fused: needs (C, Ci) = (256, 64) or (512, 128)");
  TORCH_CHECK(bits.scalar_type() == at::kByte && bits.numel() * 8 == x.numel() &&
              bits.is_contiguous(), "bits must be a contiguous uint8 [numel/8] bitmap");
  TORCH_CHECK(mean.numel() == C && invstd.numel() == C, "statistics must hold C floats");
  if (dual) {
    check_dtype(*x2, kH16, "x2");
    TORCH_CHECK(x2->sizes() == x.sizes() && x2->is_contiguous() && x2->is_cuda(), "x2 like x");
    check_aligned16(x2->data_ptr(), "x2");
    TORCH_CHECK(mean2.has_value() && invstd2.has_value() && mean2->numel() == C &&
                invstd2->numel() == C, "the shortcut BN's statistics must hold C floats");
  }
  auto f32 = x.options().dtype(at::kFloat);
  bool acc1 = false, acc1b = false, acc2 = false, acc2b = false;
  Tensor dgamma = dparam_out(dgamma_out, C, x, acc1), dbeta = dparam_out(dbeta_out, C, x, acc1b);
  TORCH_CHECK(acc1 == acc1b, "give both dgamma_out and dbeta_out");
  Tensor dg2 = dual ? dparam_out(dgamma2_out, C, x, acc2) : at::empty({0}, f32);
  Tensor db2 = dual ? dparam_out(dbeta2_out, C, x, acc2b) : at::empty({0}, f32);
  TORCH_CHECK(acc2 == acc2b, "give both dgamma2_out and dbeta2_out");
  const int64_t nb = lw::bn_reduce_blocks(M, (int)C);
  Tensor coef = at::empty({(dual ? 6 : 3) * C}, f32);
  Tensor partial = at::empty({(dual ? 2 : 1) * nb * 2 * C}, f32);
  lw::BNArgs a{}, b{};
  for (lw::BNArgs* q : {&a, &b}) {
    q->M = M;
    q->C = (int)C;
    q->bf16 = true;
    q->training = true;
    q->relu = true;
    q->coeffs_only = true;
  }
  a.accum_dparams = acc1;
  a.x = x.data_ptr();
  a.dy = dy.data_ptr();
  a.bits = ptr<uint8_t>(bits);
  a.gamma = optr<float>(weight);
  a.mean = ptr<float>(mean);
  a.invstd = ptr<float>(invstd);
  a.partial = ptr<float>(partial);
  a.dgamma = ptr<float>(dgamma);
  a.dbeta = ptr<float>(dbeta);
  a.A = ptr<float>(coef);
  a.B = a.A + C;
  a.Cc = a.A + 2 * C;
  hipStream_t st = cur_stream();
  Tensor dx2 = dual ? at::empty_like(x) : at::empty({0}, x.options());
  if (dual) {
    b.x = x2->data_ptr();
    b.gamma = optr<float>(weight2);
    b.mean = ptr<float>(*mean2);
    b.invstd = ptr<float>(*invstd2);
    b.partial = a.partial + nb * 2 * C;
    b.dgamma = ptr<float>(dg2);
    b.dbeta = ptr<float>(db2);
    b.accum_dparams = acc2;
    b.A = a.A + 3 * C;
    b.B = a.A + 4 * C;
    b.Cc = a.A + 5 * C;
    lw::bn_backward_dual(a, b, st);
  } else {
    lw::bn_backward(a, st);
  }
  Tensor o;
  const bool have_out = dw_out.has_value() && dw_out->defined();
  if (have_out) {
    o = *dw_out;
    check_dtype(o, at::kFloat, "dw_out");
    TORCH_CHECK(o.is_cuda() && o.numel() == C * Ci && o.is_contiguous(),
                "dw_out: contiguous [C][Ci] fp32");
    check_aligned16(o.data_ptr(), "dw_out");
  } else {
    o = at::zeros({C, Ci}, f32);
  }
  Tensor da2 = at::empty({M, Ci}, x.options());
  const int nblk = lw::bn3_bwd_dgemm_slabs(M, (int)C, (int)Ci);
  // one workgroup adds its dW3 into the destination itself (no slab, no reduce to defer)
  Tensor slab = nblk > 1 ? at::empty({(int64_t)nblk * C * Ci}, f32) : o;
  Tensor st2 = at::empty({s2 ? (int64_t)nblk : 0, 2, Ci}, f32);
  if (a2_from_bn2) {
    TORCH_CHECK(bn2_ss.has_value() && bn2_ss->defined() && bn2_ss->numel() == 2 * Ci,
                "a2_from_bn2 needs bn2_ss (2*Ci floats)");
    check_dtype(*bn2_ss, at::kFloat, "bn2_ss");
  }
  if (s2) {
    check_dtype(*bn2_x, kH16, "bn2_x");
    TORCH_CHECK(bn2_x->is_cuda() && bn2_x->sizes() == a2.sizes() && bn2_x->is_contiguous(),
                "bn2_x must be BN2's input [M][Ci], like a2");
    check_aligned16(bn2_x->data_ptr(), "bn2_x");
    TORCH_CHECK(bn2_ss.has_value() && bn2_ss->defined() && bn2_ss->numel() == 2 * Ci &&
                bn2_mean.has_value() && bn2_mean->defined() &&
                bn2_mean->numel() == Ci, "bn2_ss must hold 2*Ci and bn2_mean Ci floats");
    check_dtype(*bn2_ss, at::kFloat, "bn2_ss");
    check_dtype(*bn2_mean, at::kFloat, "bn2_mean");
  }
  lw::bn3_bwd_dgemm(ptr<uint16_t>(dy), ptr<uint16_t>(x), ptr<uint8_t>(bits), a.A, a.B, a.Cc,
                    ptr<uint16_t>(w3t), ptr<uint16_t>(a2), ptr<uint16_t>(da2), ptr<float>(slab),
                    M, (int)C, (int)Ci, st, dual ? ptr<uint16_t>(*x2) : nullptr,
                    dual ? b.A : nullptr,
                    dual ? b.B : nullptr, dual ? b.Cc : nullptr,
                    dual ? ptr<uint16_t>(dx2) : nullptr, nblk == 1,
                    s2 ? ptr<uint16_t>(*bn2_x) : nullptr,
                    (s2 || a2_from_bn2) ? ptr<float>(*bn2_ss) : nullptr,
                    s2 ? ptr<float>(*bn2_mean) : nullptr, s2 ? ptr<float>(st2) : nullptr,
                    a2_from_bn2);
  if (nblk > 1) {
    lw::GemmArgs g{};
    g.partial = ptr<float>(slab);
    g.C = o.data_ptr();
    g.ldc = Ci;
    g.M = (int)C;
    g.N = (int)Ci;
    g.out_bf16 = false;
    g.accumulate = have_out;
    lw::splitk_reduce(g, nblk, st);
    if (lw::splitk_take_deferred()) splitk_keep().push_back(slab);
  }
  launched("bn3_bwd_fused");
  return {da2, o, dgamma, dbeta, dx2, dg2, db2, st2};
}

// A bottleneck's BN1 backward (no downsample; bf16, training, ReLU mask from c1 through the
// forward affine scale_shift) fused with the GEMMs consuming dc1 (bnfuse.hip k_bn1_bwd_dgemm):
// reduce + finalize as bn_bwd, then dx = dc1·W1 + dy·bit3 ([M, Cin] bf16: the block's input
// gradient, its shortcut term masked by the block output's ReLU bitmap bits3) and dW1 = dc1ᵀ·x
// into dw_out (accumulated; [Wd][Cin]) or a fresh tensor. w1t = W1ᵀ [Cin][Wd].
// Returns (dx, dW1, dgamma, dbeta); dc1 is never written.
std::tuple<Tensor, Tensor, Tensor, Tensor> bn1_bwd_fused(
    Tensor da1, Tensor c1, Tensor scale_shift, c10::optional<Tensor> weight, Tensor mean,
    Tensor invstd, Tensor w1t, Tensor x, Tensor dy, Tensor bits3, c10::optional<Tensor> dw_out,
    c10::optional<Tensor> dgamma_out, c10::optional<Tensor> dbeta_out) {
  const c10::DeviceGuard guard(x.device());
  for (const Tensor* t : {&da1, &c1, &w1t, &x, &dy}) {
    check_dtype(*t, kH16, "bn1_bwd_fused operand");
    TORCH_CHECK(t->is_cuda() && t->dim() == 2 && t->is_contiguous(),
                "bn1_bwd_fused: contiguous 2-D [rows, channels] operands");
    check_aligned16(t->data_ptr(), "bn1_bwd_fused operand");
  }
  const int64_t M = c1.size(0), Wd = c1.size(1), Cin = x.size(1);
  TORCH_CHECK(da1.sizes() == c1.sizes() && x.size(0) == M && dy.sizes() == x.sizes(),
              "da1 / x / dy rows must match c1");
  TORCH_CHECK(w1t.size(0) == Cin && w1t.size(1) == Wd, "w1t must be W1ᵀ [Cin][Wd]");
  TORCH_CHECK(lw::bn1_bwd_dgemm_ok(M, (int)Wd, (int)Cin),
              "bn1_bwd_fused: needs (Wd, Cin) = (64, 256) or (128, 512)");
  TORCH_CHECK(bits3.scalar_type() == at::kByte && bits3.numel() * 8 == dy.numel() &&
              bits3.is_contiguous(), "bits3 must be a contiguous uint8 [numel/8] bitmap of dy");
  check_dtype(scale_shift, at::kFloat, "scale_shift");
  TORCH_CHECK(scale_shift.numel() == 2 * Wd && scale_shift.is_contiguous(),
              "scale_shift must hold 2*Wd floats");
  TORCH_CHECK(mean.numel() == Wd && invstd.numel() == Wd, "statistics must hold Wd floats");
  auto f32 = x.options().dtype(at::kFloat);
  bool acc1 = false, acc1b = false;
  Tensor dgamma = dparam_out(dgamma_out, Wd, x, acc1), dbeta = dparam_out(dbeta_out, Wd, x, acc1b);
  TORCH_CHECK(acc1 == acc1b, "give both dgamma_out and dbeta_out");
  Tensor coef = at::empty({3 * Wd}, f32);
  Tensor partial = at::empty({lw::bn_reduce_blocks(M, (int)Wd) * 2 * Wd}, f32);
  lw::BNArgs a{};
  a.M = M;
  a.C = (int)Wd;
  a.bf16 = true;
  a.training = true;
  a.relu = true;
  a.coeffs_only = true;
  a.accum_dparams = acc1;
  a.x = c1.data_ptr();
  a.dy = da1.data_ptr();
  a.scale = ptr<float>(scale_shift);
  a.shift = a.scale + Wd;
  a.gamma = optr<float>(weight);
  a.mean = ptr<float>(mean);
  a.invstd = ptr<float>(invstd);
  a.partial = ptr<float>(partial);
  a.dgamma = ptr<float>(dgamma);
  a.dbeta = ptr<float>(dbeta);
  a.A = ptr<float>(coef);
  a.B = a.A + Wd;
  a.Cc = a.A + 2 * Wd;
  hipStream_t st = cur_stream();
  lw::bn_backward(a, st);
  Tensor o;
  const bool have_out = dw_out.has_value() && dw_out->defined();
  if (have_out) {
    o = *dw_out;
    check_dtype(o, at::kFloat, "dw_out");
    TORCH_CHECK(o.is_cuda() && o.numel() == Wd * Cin && o.is_contiguous(),
                "dw_out: contiguous [Wd][Cin] fp32");
    check_aligned16(o.data_ptr(), "dw_out");
  } else {
    o = at::zeros({Wd, Cin}, f32);
  }
  Tensor dx = at::empty({M, Cin}, x.options());
  const int nblk = lw::bn1_bwd_dgemm_slabs(M, (int)Wd, (int)Cin);
  Tensor slab = nblk > 1 ? at::empty({(int64_t)nblk * Wd * Cin}, f32) : o;
  lw::bn1_bwd_dgemm(ptr<uint16_t>(da1), ptr<uint16_t>(c1), a.scale, a.shift, a.A, a.B, a.Cc,
                    ptr<uint16_t>(w1t), ptr<uint16_t>(x), ptr<uint16_t>(dy), ptr<uint8_t>(bits3),
                    ptr<uint16_t>(dx), ptr<float>(slab), M, (int)Wd, (int)Cin, nblk == 1, st);
  if (nblk > 1) {
    lw::GemmArgs g{};
    g.partial = ptr<float>(slab);
    g.C = o.data_ptr();
    g.ldc = Cin;
    g.M = (int)Wd;
    g.N = (int)Cin;
    g.out_bf16 = false;
    g.accumulate = have_out;
    lw::splitk_reduce(g, nblk, st);
    if (lw::splitk_take_deferred()) splitk_keep().push_back(slab);
  }
  launched("bn1_bwd_fused");
  return {dx, o, dgamma, dbeta};
}

// Weight gradient of the tap-reuse conv (conv3tap.hip k_conv3_tap_wgrad): dy [N, Co, H, W] and
// x [N, C, H, W] bf16 channels_last; returns fp32 dW in [Co][3][3][C] memory order (a channels_last
// [Co, C, 3, 3] tensor), written into / accumulated onto `out` when given.
Tensor conv3_tap_wgrad(Tensor dy, Tensor x, c10::optional<Tensor> out, bool accumulate) {
  const c10::DeviceGuard guard(x.device());
  check_dtype(x, kH16, "x");
  check_dtype(dy, kH16, "dy");
  TORCH_CHECK(x.is_cuda() && dy.is_cuda() && x.dim() == 4 && dy.dim() == 4 &&
              x.is_contiguous(at::MemoryFormat::ChannelsLast) &&
              dy.is_contiguous(at::MemoryFormat::ChannelsLast), "x, dy: channels_last 4-D");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), Co = dy.size(1);
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == H && dy.size(3) == W, "dy / x shapes");
  TORCH_CHECK(lw::conv3_tap_ok((int)C, (int)Co, (int)H, (int)W), "conv3_tap_wgrad: geometry");
  TORCH_CHECK(x.numel() * 2 < (1LL << 31) && dy.numel() * 2 < (1LL << 31), "operand > 2 GiB");
  check_aligned16(x.data_ptr(), "x");
  check_aligned16(dy.data_ptr(), "dy");
  Tensor o;
  if (out.has_value() && out->defined()) {
    o = *out;
    check_dtype(o, at::kFloat, "out");
    TORCH_CHECK(o.is_cuda() && o.numel() == Co * 9 * C, "out: Co*9*C floats");
    TORCH_CHECK(o.is_contiguous() || o.is_contiguous(at::MemoryFormat::ChannelsLast),
                "out: dense [Co][3][3][C] memory");
    if (o.dim() == 4) TORCH_CHECK(o.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                                  o.size(1) == C && o.size(2) == 3, "out: channels_last [Co, C, 3, 3]");
    check_aligned16(o.data_ptr(), "out");
  } else {
    o = at::empty({Co, C, 3, 3}, x.options().dtype(at::kFloat).memory_format(at::MemoryFormat::ChannelsLast));
    accumulate = false;
  }
  const int splits = lw::conv3_tap_wgrad_splits((int)N, (int)H, (int)W, (int)C, (int)Co);
  Tensor part = at::empty({(int64_t)splits * Co * 9 * C}, x.options().dtype(at::kFloat));
  lw::conv3_tap_wgrad(ptr<uint16_t>(dy), ptr<uint16_t>(x), ptr<float>(part),
                      static_cast<float*>(o.data_ptr()), (int)N, (int)H, (int)W, (int)C, (int)Co,
                      accumulate ? 1 : 0, cur_stream());
  launched("conv3_tap_wgrad");
  return o;
}

// ---------------------------------------------------------------- BN pieces for fused blocks
// Batch statistics of x ([M, C] / channels_last), or — with `stats` [2, C, nb] from a GEMM's
// column-statistics epilogue — only the finalize. Returns (mean, invstd, scale_shift[2C]).
std::tuple<Tensor, Tensor, Tensor> bn_stats(Tensor x, c10::optional<Tensor> stats,
                                            c10::optional<Tensor> weight,
                                            c10::optional<Tensor> bias,
                                            c10::optional<Tensor> rmean,
                                            c10::optional<Tensor> rvar, double momentum,
                                            double eps) {
  const c10::DeviceGuard guard(x.device());
  check_nhwc(x, "x");
  const int64_t C = x.dim() == 4 ? x.size(1) : x.size(-1);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= kMaxBnC, "bn_stats needs C % 8 == 0 and C <= ", kMaxBnC);
  auto f32 = x.options().dtype(at::kFloat);
  Tensor mean = at::empty({C}, f32), invstd = at::empty({C}, f32);
  Tensor ss = at::empty({2 * C}, f32);
  lw::BNArgs a{};
  a.x = x.data_ptr();
  a.M = M;
  a.C = (int)C;
  a.bf16 = x.scalar_type() == kH16;
  a.training = true;
  a.eps = (float)eps;
  a.momentum = (float)momentum;
  a.gamma = optr<float>(weight);
  a.beta = optr<float>(bias);
  a.rmean = optr<float>(rmean);
  a.rvar = optr<float>(rvar);
  a.mean = ptr<float>(mean);
  a.invstd = ptr<float>(invstd);
  a.scale = ptr<float>(ss);
  a.shift = a.scale + C;
  Tensor partial;
  if (stats.has_value() && stats->defined()) {
    check_dtype(*stats, at::kFloat, "stats");
    TORCH_CHECK(stats->dim() == 3 && stats->size(1) == 2 && stats->size(2) == C &&
                stats->is_contiguous(), "stats must be a contiguous [rows, 2, C] tensor");
    const int64_t R = stats->size(0);
    partial = at::empty({(int64_t)lw::colsum_blocks(R) * 2 * C}, f32);
    a.partial = ptr<float>(partial);
    a.stat_rows = ptr<float>(*stats);
    a.stats_rows_n = R;
  } else {
    partial = at::empty({(int64_t)lw::bn_reduce_blocks(M, (int)C) * 2 * C}, f32);
    a.partial = ptr<float>(partial);
  }
  lw::bn_stats(a, cur_stream());
  launched("bn_stats");
  return {mean, invstd, ss};
}

// fused stem BN-apply + ReLU + max-pool (bn.hip)
static void stem_geom(const Tensor& x, int64_t k, int64_t s, int64_t p, lw::StemArgs& a) {
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem input must be channels_last 4-D");
  check_dtype(x, kH16, "x");
  a.N = (int)x.size(0); a.C = (int)x.size(1); a.H = (int)x.size(2); a.W = (int)x.size(3);
  TORCH_CHECK(a.C % 8 == 0 && a.C <= kMaxBnC, "stem pool needs C % 8 == 0 and C <= ", kMaxBnC);
  // PyTorch semantics: padding at most half the window (no window lies entirely in padding)
  TORCH_CHECK(k >= 1 && k * k <= 255 && s >= 1 && p >= 0 && 2 * p <= k, "pool geometry");
  a.k = (int)k; a.s = (int)s; a.p = (int)p;
  a.Ho = (int)((a.H + 2 * p - k) / s + 1);
  a.Wo = (int)((a.W + 2 * p - k) / s + 1);
  // the kernels decompose flat pixel / output indices in 32-bit arithmetic
  TORCH_CHECK((int64_t)a.N * a.H * a.W < (1LL << 31) &&
              (int64_t)a.N * a.Ho * a.Wo * (a.C / 8) < (1LL << 31), "stem pool: tensor too large");
}

// the forward pass on geometry `a` with BN coefficients `scale` / `shift` ([C] each)
static std::tuple<Tensor, Tensor> pool_fwd_launch(const Tensor& x, lw::StemArgs& a,
                                                  const float* scale, const float* shift) {
  Tensor out = at::empty({a.N, a.C, a.Ho, a.Wo},
                         x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor idx = at::empty({(int64_t)a.N * a.Ho * a.Wo * a.C}, x.options().dtype(at::kByte));
  a.x = x.data_ptr();
  a.scale = scale;
  a.shift = shift;
  a.out = out.data_ptr();
  a.idx = ptr<uint8_t>(idx);
  lw::stem_pool_fwd(a, cur_stream());
  launched("stem_pool_fwd");
  return {out, idx};
}

std::tuple<Tensor, Tensor> stem_pool_fwd(Tensor x, Tensor scale_shift, int64_t k, int64_t s,
                                         int64_t p) {
  const c10::DeviceGuard guard(x.device());
  lw::StemArgs a{};
  stem_geom(x, k, s, p, a);
  check_dtype(scale_shift, at::kFloat, "scale_shift");
  TORCH_CHECK(scale_shift.numel() == 2 * a.C && scale_shift.is_contiguous(), "scale_shift");
  return pool_fwd_launch(x, a, ptr<float>(scale_shift), ptr<float>(scale_shift) + a.C);
}

// max-pool of a post-ReLU 16-bit map (no BN): scale / A = 1, shift / B / C = 0, read from the
// device-resident [ones][zeros] table (bn.hip kPoolIdentity) instead of filled per call
static const float* pool_ones(int64_t C) {
  const float* base = lw::pool_identity_consts();
  TORCH_CHECK(base != nullptr && C <= lw::kPoolIdC, "pool identity constants unavailable");
  return base + (lw::kPoolIdC - C);           // C ones, then the zeros
}

std::tuple<Tensor, Tensor> relu_pool_fwd(Tensor x, int64_t k, int64_t s, int64_t p) {
  const c10::DeviceGuard guard(x.device());
  lw::StemArgs a{};
  stem_geom(x, k, s, p, a);
  const float* ones = pool_ones(a.C);
  return pool_fwd_launch(x, a, ones, ones + a.C);
}

Tensor relu_pool_bwd(Tensor dp, Tensor idx, Tensor x, int64_t k, int64_t s, int64_t p) {
  const c10::DeviceGuard guard(x.device());
  lw::StemArgs a{};
  stem_geom(x, k, s, p, a);
  check_dtype(dp, kH16, "dp");
  TORCH_CHECK(dp.is_contiguous(at::MemoryFormat::ChannelsLast) && dp.size(2) == a.Ho &&
              dp.size(3) == a.Wo && dp.size(1) == a.C && dp.size(0) == a.N, "dp shape/layout");
  TORCH_CHECK(idx.numel() == dp.numel() && idx.scalar_type() == at::kByte, "idx");
  const float* ones = pool_ones(a.C);
  const float* zeros = ones + a.C;
  Tensor dx = at::empty_like(x);
  a.x = x.data_ptr();
  a.dp = dp.data_ptr();
  a.idx = ptr<uint8_t>(idx);
  a.dx = dx.data_ptr();
  a.scale = ones;
  a.shift = zeros;
  a.mean = zeros;                   // unused by the apply pass
  a.A = const_cast<float*>(ones);   // (read-only here: relu_pool_bwd only applies them)
  a.B = const_cast<float*>(zeros);
  a.Cc = const_cast<float*>(zeros);
  lw::relu_pool_bwd(a, cur_stream());
  launched("relu_pool_bwd");
  return dx;
}

std::tuple<Tensor, Tensor, Tensor> stem_pool_bwd(Tensor dp, Tensor idx, Tensor x,
                                                 Tensor scale_shift, c10::optional<Tensor> weight,
                                                 Tensor mean, Tensor invstd, int64_t k, int64_t s,
                                                 int64_t p, c10::optional<Tensor> dgamma_out,
                                                 c10::optional<Tensor> dbeta_out,
                                                 c10::optional<Tensor> pooled) {
  const c10::DeviceGuard guard(x.device());
  lw::StemArgs a{};
  stem_geom(x, k, s, p, a);
  check_dtype(dp, kH16, "dp");
  TORCH_CHECK(dp.is_contiguous(at::MemoryFormat::ChannelsLast) && dp.size(2) == a.Ho &&
              dp.size(3) == a.Wo && dp.size(1) == a.C && dp.size(0) == a.N, "dp shape/layout");
  TORCH_CHECK(idx.numel() == dp.numel() && idx.scalar_type() == at::kByte, "idx");
  if (pooled.has_value() && pooled->defined()) {
    check_dtype(*pooled, kH16, "pooled");
    TORCH_CHECK(pooled->sizes() == dp.sizes() &&
                pooled->is_contiguous(at::MemoryFormat::ChannelsLast), "pooled shape/layout");
    a.pooled = pooled->data_ptr();
  }
  auto f32 = x.options().dtype(at::kFloat);
  Tensor dx = at::empty_like(x);
  bool accum = false;
  Tensor dgamma = dparam_out(dgamma_out, a.C, x, accum);
  Tensor dbeta = dparam_out(dbeta_out, a.C, x, accum);
  a.accum_dparams = accum;
  Tensor coef = at::empty({3 * a.C}, f32);
  Tensor partial = at::empty({(int64_t)lw::bn_reduce_blocks((int64_t)a.N * a.H * a.W, a.C) * 2 * a.C}, f32);
  a.x = x.data_ptr();
  a.dp = dp.data_ptr();
  a.idx = ptr<uint8_t>(idx);
  a.dx = dx.data_ptr();
  a.scale = ptr<float>(scale_shift);
  a.shift = a.scale + a.C;
  a.gamma = optr<float>(weight);
  a.mean = ptr<float>(mean);
  a.invstd = ptr<float>(invstd);
  a.partial = ptr<float>(partial);
  a.dgamma = ptr<float>(dgamma);
  a.dbeta = ptr<float>(dbeta);
  a.A = ptr<float>(coef);
  a.B = a.A + a.C;
  a.Cc = a.A + 2 * a.C;
  lw::stem_pool_bwd(a, cur_stream());
  launched("stem_pool_bwd");
  return {dx, dgamma, dbeta};
}

// The stem backward with its pool/BN apply fused into the 7x7/2 conv's weight gradient
// (stemfuse.hip): pooled-side statistics + finalize as stem_pool_bwd, then one kernel forms the
// conv-output gradient tile by tile in LDS and accumulates dW against the 4-channel image x4
// ([N, 4, 2H, 2W] channels_last). Returns (dW [64][7 * 8 * 4] fp32 — [co][r][s][ci], tap 7 and
// channel 3 padding — dgamma, dbeta); the conv-output gradient is never written.
std::tuple<Tensor, Tensor, Tensor> stem_bwd_fused(Tensor dp, Tensor idx, Tensor x,
                                                  Tensor scale_shift, c10::optional<Tensor> weight,
                                                  Tensor mean, Tensor invstd, int64_t k, int64_t s,
                                                  int64_t p, c10::optional<Tensor> dgamma_out,
                                                  c10::optional<Tensor> dbeta_out, Tensor pooled,
                                                  Tensor x4) {
  const c10::DeviceGuard guard(x.device());
  lw::StemArgs a{};
  stem_geom(x, k, s, p, a);
  check_dtype(dp, kH16, "dp");
  TORCH_CHECK(dp.is_contiguous(at::MemoryFormat::ChannelsLast) && dp.size(2) == a.Ho &&
              dp.size(3) == a.Wo && dp.size(1) == a.C && dp.size(0) == a.N, "dp shape/layout");
  TORCH_CHECK(idx.numel() == dp.numel() && idx.scalar_type() == at::kByte, "idx");
  check_dtype(pooled, kH16, "pooled");
  TORCH_CHECK(pooled.sizes() == dp.sizes() &&
              pooled.is_contiguous(at::MemoryFormat::ChannelsLast), "pooled shape/layout");
  check_dtype(x4, kH16, "x4");
  TORCH_CHECK(x4.dim() == 4 && x4.size(0) == a.N && x4.size(1) == 4 &&
              x4.is_contiguous(at::MemoryFormat::ChannelsLast), "x4: [N, 4, H, W] channels_last");
  TORCH_CHECK(k == 3 && s == 2 && p == 1 &&
              lw::stem_bwd_wgrad_ok(a.C, a.H, a.W, a.Ho, a.Wo, (int)x4.size(2), (int)x4.size(3)),
              "stem_bwd_fused: 64 channels at 112x112 from a 224x224 image, 3x3/2/1 pool");
  TORCH_CHECK(x4.numel() * 2 < (1LL << 31), "x4 > 2 GiB");
  check_aligned16(x4.data_ptr(), "x4");
  auto f32 = x.options().dtype(at::kFloat);
  bool accum = false;
  Tensor dgamma = dparam_out(dgamma_out, a.C, x, accum);
  Tensor dbeta = dparam_out(dbeta_out, a.C, x, accum);
  a.accum_dparams = accum;
  a.coeffs_only = true;
  a.pooled = pooled.data_ptr();
  Tensor coef = at::empty({3 * a.C}, f32);
  Tensor partial = at::empty({(int64_t)lw::bn_reduce_blocks((int64_t)a.N * a.H * a.W, a.C) * 2 * a.C}, f32);
  a.x = x.data_ptr();
  a.dp = dp.data_ptr();
  a.idx = ptr<uint8_t>(idx);
  a.scale = ptr<float>(scale_shift);
  a.shift = a.scale + a.C;
  a.gamma = optr<float>(weight);
  a.mean = ptr<float>(mean);
  a.invstd = ptr<float>(invstd);
  a.partial = ptr<float>(partial);
  a.dgamma = ptr<float>(dgamma);
  a.dbeta = ptr<float>(dbeta);
  a.A = ptr<float>(coef);
  a.B = a.A + a.C;
  a.Cc = a.A + 2 * a.C;
  hipStream_t st = cur_stream();
  lw::stem_pool_bwd(a, st);
  const int nblk = lw::stem_bwd_wgrad_blocks(a.N, a.Ho);
  Tensor slab = at::empty({(int64_t)nblk * 64 * 224}, f32);
  Tensor o = at::empty({64, 224}, f32);
  lw::stem_bwd_wgrad(static_cast<const uint16_t*>(a.dp), a.idx, ptr<uint16_t>(x), a.scale,
                     a.shift, a.A, a.B, a.Cc, ptr<uint16_t>(x4), ptr<float>(slab), a.N, a.Ho,
                     a.Wo, (int)x4.size(2), (int)x4.size(3), st);
  lw::GemmArgs g{};
  g.partial = ptr<float>(slab);
  g.C = o.data_ptr();
  g.ldc = 224;
  g.M = 64;
  g.N = 224;
  g.out_bf16 = false;
  g.accumulate = false;
  lw::splitk_reduce(g, nblk, st);
  if (lw::splitk_take_deferred()) splitk_keep().push_back(slab);
  launched("stem_bwd_fused");
  return {o, dgamma, dbeta};
}

// y = relu?(x*scale+shift [+ res | + res*rscale+rshift])
Tensor bn_apply(Tensor x, Tensor scale_shift, c10::optional<Tensor> res,
                c10::optional<Tensor> res_scale_shift, bool relu,
                c10::optional<Tensor> bits_out) {
  const c10::DeviceGuard guard(x.device());
  check_nhwc(x, "x");
  const int64_t C = x.dim() == 4 ? x.size(1) : x.size(-1);
  TORCH_CHECK(C % 8 == 0 && C <= kMaxBnC, "bn_apply needs C % 8 == 0 and C <= ", kMaxBnC);
  check_dtype(scale_shift, at::kFloat, "scale_shift");
  TORCH_CHECK(scale_shift.numel() == 2 * C && scale_shift.is_contiguous(), "scale_shift size");
  Tensor y = at::empty_like(x);
  lw::BNArgs a{};
  a.x = x.data_ptr();
  a.y = y.data_ptr();
  a.M = x.numel() / C;
  a.C = (int)C;
  a.bf16 = x.scalar_type() == kH16;
  a.relu = relu;
  a.scale = ptr<float>(scale_shift);
  a.shift = a.scale + C;
  if (bits_out.has_value() && bits_out->defined()) {
    TORCH_CHECK(relu, "a ReLU bitmap needs relu=True");
    TORCH_CHECK(bits_out->scalar_type() == at::kByte && bits_out->numel() * 8 == x.numel() &&
                bits_out->is_contiguous(), "bits_out must be a contiguous uint8 [numel/8]");
    a.bits = ptr<uint8_t>(*bits_out);
  }
  if (res.has_value() && res->defined()) {
    check_nhwc(*res, "res");
    TORCH_CHECK(res->numel() == x.numel() && res->scalar_type() == x.scalar_type(),
                "residual must match x");
    a.res = res->data_ptr();
    if (res_scale_shift.has_value() && res_scale_shift->defined()) {
      check_dtype(*res_scale_shift, at::kFloat, "res_scale_shift");
      TORCH_CHECK(res_scale_shift->numel() == 2 * C && res_scale_shift->is_contiguous(),
                  "res_scale_shift size");
      a.res_scale = ptr<float>(*res_scale_shift);
      a.res_shift = a.res_scale + C;
    }
  }
  lw::bn_apply(a, cur_stream());
  launched("bn_apply");
  return y;
}

// test hook: a deliberately invalid launch (block of 2048 threads) must raise in launched()
void selftest_bad_launch(Tensor any) {
  const c10::DeviceGuard guard(any.device());
  lw::launch_invalid_config_for_test(cur_stream());
  launched("selftest_bad_launch");
}

// test hook: keep the current stream busy for `ms` milliseconds (bounded, always drains)
void selftest_spin(Tensor any, double ms) {
  const c10::DeviceGuard guard(any.device());
  lw::spin_for_test(ms, cur_stream());
  launched("selftest_spin");
}

}  // namespace

LW_LIBRARY(LW_OPS_NS, m) {
  m.def("workspace_bytes(int n_small, int n_large, int n_tasks) -> int", &workspace_bytes);
  m.def("selftest_bad_launch(Tensor any) -> ()");
  m.def("selftest_spin(Tensor any, float ms) -> ()");
  m.def(
      "select_compress(Tensor(a!) g, Tensor(b!)? ef, Tensor seg_off, Tensor seg_n, Tensor keep, "
      "Tensor cap_off, Tensor small_segs, Tensor large_segs, Tensor tasks, Tensor task_lo, "
      "Tensor(c!) ws, int km, int out, Tensor(d!)? pairs, Tensor(e!)? vals, Tensor(f!)? idx, "
      "int gid_base, int step, int seed, Tensor? step_t=None, Tensor(g!)? overflow=None, "
      "Tensor(h!)? mom=None, bool staged=False, int max_seg_tasks=0, Tensor? mc_p=None, "
      "Tensor? mc_wd=None, float mc=0.0, float mc_wmul=1.0) -> ()");
  m.def(
      "select_stage(Tensor(a!) g, Tensor(b!)? ef, Tensor seg_off, Tensor seg_n, Tensor keep, "
      "Tensor cap_off, Tensor small_segs, Tensor large_segs, Tensor tasks, Tensor task_lo, "
      "Tensor(c!) ws, int km, int t_lo, int t_hi, bool zero, int gid_base, int step, int seed, "
      "Tensor? step_t=None) -> ()");
  m.def(
      "quant_stage(Tensor(a!) g, Tensor(b!)? ef, Tensor seg_off, Tensor seg_n, Tensor segs, "
      "Tensor tasks, Tensor task_lo, Tensor rec_off, Tensor(c!) ws, int qstates, int t_lo, "
      "int t_hi) -> ()");
  m.def(
      "thresh_count(Tensor(a!) g, Tensor(b!)? ef, Tensor seg_off, Tensor seg_n, Tensor large_segs, "
      "Tensor tasks, Tensor task_lo, Tensor(c!) ws, float V, int adaptive, Tensor(d!) counts_out) "
      "-> ()");
  m.def(
      "thresh_dense(Tensor(a!) g, Tensor(b!)? ef, Tensor seg_off, Tensor seg_n, Tensor large_segs, "
      "Tensor tasks, Tensor task_lo, Tensor(c!) ws, float V, int adaptive) -> ()");
  m.def(
      "thresh_write(Tensor(a!) g, Tensor(b!)? ef, Tensor seg_off, Tensor seg_n, Tensor cap_off, "
      "Tensor large_segs, Tensor tasks, Tensor task_lo, Tensor(c!) ws, Tensor(d!) pairs, "
      "Tensor(e!)? overflow=None) -> ()");
  m.def(
      "unpack_pairs(Tensor gathered, int world, Tensor(a!) g, Tensor seg_off, Tensor seg_n, "
      "Tensor cap_off, Tensor utasks) -> ()");
  m.def(
      "unpack_pairs_sgd(Tensor gathered, int world, Tensor seg_off, Tensor cap_off, "
      "Tensor ftasks, Tensor(a!) p, Tensor(b!) buf, Tensor seg_wd, float lr, float momentum, "
      "float dampening, int nesterov, int first_step, float grad_scale, Tensor? hyper, "
      "Tensor(c!)? pb) -> ()");
  m.def(
      "unpack_validx(Tensor vals, Tensor idx, Tensor slot_seg, int world, Tensor(a!) g, "
      "Tensor seg_off) -> ()");
  m.def(
      "quantize(Tensor(a!) g, Tensor(b!)? ef, Tensor seg_off, Tensor seg_n, Tensor segs, "
      "Tensor tasks, Tensor task_lo, Tensor rec_off, Tensor(c!) ws, Tensor(d!) payload, int q, "
      "int qstates, int gid_base, int step, int tag, int seed, Tensor? step_t=None, "
      "bool staged=False) -> ()");
  m.def(
      "dequantize(Tensor gathered, int world, Tensor(a!) g, Tensor seg_off, Tensor seg_n, "
      "Tensor segs, Tensor tasks, Tensor task_lo, Tensor rec_off, int q, int qstates) -> ()");
  m.def(
      "dequant_shard(Tensor recv, int world, int hdr, Tensor gtab, int g0, int ng, int q, "
      "int qstates, Tensor(a!) out) -> ()");
  m.def("bf16_expand(Tensor x, Tensor(a!) out) -> ()");
  m.def("wire_wait(Tensor dev, float us, int nwg) -> ()");
  m.def(
      "mc_prep(Tensor(a!) g, Tensor(b!) u, Tensor? p, Tensor seg_off, Tensor seg_n, Tensor segs, "
      "Tensor tasks, Tensor? seg_wd, float mc, float wmul) -> ()");
  m.def("mc_mask(Tensor(a!) u, Tensor e) -> ()");
  m.def("step_bump(Tensor(a!) c) -> ()");
  m.def("splitk_defer(Tensor dev, bool on) -> ()");
  m.def("xent_mean(Tensor rows, Tensor target, int ignore_index) -> (Tensor, Tensor)");
  m.def("pack_kc_multi(Tensor[] w, Tensor(a!)[] out, int[] prm) -> ()");
  m.def("xent_scale(Tensor grad, Tensor gl, Tensor n) -> Tensor");
  m.def("splitk_flush(Tensor dev) -> int");
  m.def("splitk_discard(Tensor dev) -> int");
  m.def("splitk_pending() -> int", &splitk_pending);
  m.def(
      "sgd_step(Tensor(a!) p, Tensor g, Tensor(b!) buf, Tensor seg_off, Tensor seg_n, "
      "Tensor segs, Tensor tasks, Tensor seg_wd, float lr, float momentum, float dampening, "
      "int nesterov, int first_step, float grad_scale, Tensor? hyper=None, "
      "Tensor(c!)? pb=None) -> ()");
  m.def("normalize_u8(Tensor input, Tensor(a!) out, float[] mean, float[] std) -> ()");
  m.def("cifar_augment(Tensor data, Tensor idx, Tensor prm, int offset, int crop, int cutout, "
        "Tensor(a!) out) -> ()");
  m.def("gap_fwd(Tensor x) -> Tensor");
  m.def("sum_repeats(Tensor w, int R) -> Tensor");
  m.def("repeat_store(Tensor g, Tensor(a!) out, int R, bool accumulate) -> ()");
  m.def("pack_dgrad_nkc(Tensor w, int[] cls, int sh, int sw) -> Tensor");
  m.def("relu_bias_bwd(Tensor dy, Tensor? y, Tensor(a!)? db_out) -> (Tensor, Tensor)");
  m.def("xent(Tensor logits, Tensor target, float gscale, int ignore_index, bool want_grad) "
        "-> (Tensor, Tensor, Tensor)");
  m.def("gap_bwd(Tensor dy, int H, int W) -> Tensor");
  m.def(
      "bn_fwd(Tensor x, Tensor? res, Tensor? weight, Tensor? bias, Tensor(a!)? running_mean, "
      "Tensor(b!)? running_var, bool training, float momentum, float eps, bool relu) "
      "-> (Tensor, Tensor, Tensor, Tensor)");
  m.def(
      "bn_bwd(Tensor dy, Tensor x, Tensor? y, Tensor? weight, Tensor mean, Tensor invstd, "
      "Tensor? scale_shift, bool training, bool relu, bool need_dres, Tensor? bits=None, "
      "Tensor(a!)? dgamma_out=None, Tensor(b!)? dbeta_out=None, Tensor? stats_rows=None) "
      "-> (Tensor, Tensor, Tensor, Tensor)");
  m.def("stem_conv7(Tensor x, Tensor w) -> (Tensor, Tensor)");
  m.def("conv3_tap(Tensor x, Tensor w, int Co, bool want_stats) -> (Tensor, Tensor)");
  m.def("bn3_bwd_fused(Tensor dy, Tensor x, Tensor bits, Tensor? weight, Tensor mean, "
        "Tensor invstd, Tensor w3t, Tensor a2, Tensor(a!)? dw_out, Tensor(b!)? dgamma_out, "
        "Tensor(c!)? dbeta_out, Tensor? x2=None, Tensor? weight2=None, Tensor? mean2=None, "
        "Tensor? invstd2=None, Tensor(d!)? dgamma2_out=None, Tensor(e!)? dbeta2_out=None, "
        "Tensor? bn2_x=None, Tensor? bn2_ss=None, Tensor? bn2_mean=None, "
        "bool a2_from_bn2=False) -> (Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("stem_bwd_fused(Tensor dp, Tensor idx, Tensor x, Tensor scale_shift, Tensor? weight, "
        "Tensor mean, Tensor invstd, int k, int s, int p, Tensor(a!)? dgamma_out, "
        "Tensor(b!)? dbeta_out, Tensor pooled, Tensor x4) -> (Tensor, Tensor, Tensor)");
  m.def("bn1_bwd_fused(Tensor da1, Tensor c1, Tensor scale_shift, Tensor? weight, Tensor mean, "
        "Tensor invstd, Tensor w1t, Tensor x, Tensor dy, Tensor bits3, Tensor(a!)? dw_out, "
        "Tensor(b!)? dgamma_out, Tensor(c!)? dbeta_out) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("conv3_tap_wgrad(Tensor dy, Tensor x, Tensor(a!)? out, bool accumulate) -> Tensor");
  m.def(
      "bn_bwd_dual(Tensor dy, Tensor x, Tensor x2, Tensor bits, Tensor? weight, Tensor mean, "
      "Tensor invstd, Tensor? weight2, Tensor mean2, Tensor invstd2, "
      "Tensor(a!)? dgamma_out=None, Tensor(b!)? dbeta_out=None, Tensor(c!)? dgamma2_out=None, "
      "Tensor(d!)? dbeta2_out=None) -> (Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def(
      "gemm(Tensor A, int lda, bool a_kcontig, Tensor B, int ldb, bool b_kcontig, int M, int N, "
      "int K, Tensor? bias, bool relu, int splits, bool out_bf16) -> Tensor");
  m.def(
      "gemm_ex(Tensor A, int lda, bool a_kcontig, Tensor B, int ldb, bool b_kcontig, int M, "
      "int N, int K, Tensor? bias, bool relu, int splits, bool out_bf16, int tile, "
      "Tensor? pro_scale, Tensor? pro_shift, bool pro_on_a, bool want_stats, "
      "Tensor(a!)? out=None, Tensor? addend=None, bool accumulate=False, int ldc=0, "
      "Tensor? addend_bits=None, Tensor? bst_x=None, Tensor? bst_mean=None, "
      "Tensor? bst_scale_shift=None, Tensor? bst_bits=None) "
      "-> (Tensor, Tensor)");
  m.def("pack_dgrad_kc(Tensor w, int[] cls, int sh, int sw, int kmax) -> Tensor");
  m.def(
      "conv_ex(Tensor G, Tensor Op, int mode, int[] geom, int N, int tile, int splits, "
      "bool out_bf16, Tensor? pro_scale, Tensor? pro_shift, bool want_stats, Tensor(a!)? out, "
      "bool accumulate, int ldc, bool b_kcontig, int ldb, Tensor? addend=None, "
      "Tensor? bst_x=None, Tensor? bst_mean=None, Tensor? bst_scale_shift=None, "
      "Tensor? bst_bits=None, Tensor? bias=None, bool relu=False) -> (Tensor, Tensor)");
  m.def(
      "bn_stats(Tensor x, Tensor? stats, Tensor? weight, Tensor? bias, Tensor(a!)? running_mean, "
      "Tensor(b!)? running_var, float momentum, float eps) -> (Tensor, Tensor, Tensor)");
  m.def("bn_apply(Tensor x, Tensor scale_shift, Tensor? res, Tensor? res_scale_shift, bool relu, "
        "Tensor(a!)? bits_out=None) -> Tensor");
  m.def("stem_pool_fwd(Tensor x, Tensor scale_shift, int k, int s, int p) -> (Tensor, Tensor)");
  m.def("relu_pool_fwd(Tensor x, int k, int s, int p) -> (Tensor, Tensor)");
  m.def("relu_pool_bwd(Tensor dp, Tensor idx, Tensor x, int k, int s, int p) -> Tensor");
  m.def(
      "stem_pool_bwd(Tensor dp, Tensor idx, Tensor x, Tensor scale_shift, Tensor? weight, "
      "Tensor mean, Tensor invstd, int k, int s, int p, Tensor(a!)? dgamma_out=None, "
      "Tensor(b!)? dbeta_out=None, Tensor? pooled=None) -> (Tensor, Tensor, Tensor)");
}

LW_LIBRARY_IMPL(LW_OPS_NS, CUDA, m) {
  m.impl("selftest_bad_launch", &selftest_bad_launch);
  m.impl("selftest_spin", &selftest_spin);
  m.impl("select_compress", &select_compress);
  m.impl("select_stage", &select_stage);
  m.impl("quant_stage", &quant_stage);
  m.impl("thresh_count", &thresh_count);
  m.impl("thresh_write", &thresh_write);
  m.impl("thresh_dense", &thresh_dense);
  m.impl("unpack_pairs", &unpack_pairs);
  m.impl("unpack_pairs_sgd", &unpack_pairs_sgd);
  m.impl("unpack_validx", &unpack_validx);
  m.impl("quantize", &quantize);
  m.impl("dequantize", &dequantize);
  m.impl("dequant_shard", &dequant_shard);
  m.impl("bf16_expand", &bf16_expand);
  m.impl("wire_wait", &wire_wait);
  m.impl("sgd_step", &sgd_step);
  m.impl("mc_prep", &mc_prep);
  m.impl("mc_mask", &mc_mask);
  m.impl("step_bump", &step_bump);
  m.impl("splitk_defer", &splitk_defer);
  m.impl("xent_mean", &xent_mean);
  m.impl("pack_kc_multi", &pack_kc_multi);
  m.impl("xent_scale", &xent_scale);
  m.impl("splitk_flush", &splitk_flush);
  m.impl("splitk_discard", &splitk_discard);
  m.impl("normalize_u8", &normalize_u8);
  m.impl("cifar_augment", &cifar_augment);
  m.impl("gap_fwd", &gap_fwd);
  m.impl("sum_repeats", &sum_repeats);
  m.impl("repeat_store", &repeat_store);
  m.impl("pack_dgrad_nkc", &pack_dgrad_nkc);
  m.impl("relu_bias_bwd", &relu_bias_bwd);
  m.impl("xent", &xent);
  m.impl("gap_bwd", &gap_bwd);
  m.impl("bn_fwd", &bn_fwd);
  m.impl("bn_bwd", &bn_bwd);
  m.impl("bn_bwd_dual", &bn_bwd_dual);
  m.impl("stem_conv7", &stem_conv7);
  m.impl("conv3_tap", &conv3_tap);
  m.impl("conv3_tap_wgrad", &conv3_tap_wgrad);
  m.impl("bn3_bwd_fused", &bn3_bwd_fused);
  m.impl("bn1_bwd_fused", &bn1_bwd_fused);
  m.impl("stem_bwd_fused", &stem_bwd_fused);
  m.impl("gemm", &gemm);
  m.impl("gemm_ex", &gemm_ex);
  m.impl("conv_ex", &conv_ex);
  m.impl("pack_dgrad_kc", &pack_dgrad_kc);
  m.impl("bn_stats", &bn_stats);
  m.impl("bn_apply", &bn_apply);
  m.impl("stem_pool_fwd", &stem_pool_fwd);
  m.impl("relu_pool_fwd", &relu_pool_fwd);
  m.impl("relu_pool_bwd", &relu_pool_bwd);
  m.impl("stem_pool_bwd", &stem_pool_bwd);
}
