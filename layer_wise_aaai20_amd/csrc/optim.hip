// Fused multi-tensor SGD (momentum / Nesterov / weight decay / dampening / grad unscale) over the
// flat parameter, gradient and momentum arenas: ONE launch updates the whole model.
// Semantics are those of torch.optim.SGD, which the reference uses for both workloads
// (CIFAR10/torch_backend.py:120-143, IMAGENET/training/train_imagenet_nv.py:188-191), with the
// fp16 master-gradient unscale of train_imagenet_nv.py:424-426 folded in as `grad_scale`, and the
// master -> model copy of fp16util.py:103-138 (master_params_to_model_params) folded in as the
// bf16 mirror write `pb`: the next forward reads the mirror with no cast pass.
#include "common.h"
#include "lw_kernels.h"
#include "elem16.h"
#include "sgd_elem.h"

namespace lw {

constexpr int SNT = 256;
constexpr int SEPB = kLargeEPB;


template <bool MOM, bool NEST, bool FIRST>
__global__ __launch_bounds__(SNT) void k_sgd(float* __restrict__ p, const float* __restrict__ g,
                                             float* __restrict__ buf,
                                             const int64_t* __restrict__ seg_off,
                                             const int32_t* __restrict__ seg_n,
                                             const int32_t* __restrict__ segs,
                                             const int2* __restrict__ tasks,
                                             const float* __restrict__ seg_wd, float lr,
                                             float momentum, float dampening, float grad_scale,
                                             const float* __restrict__ hyper,
                                             uint16_t* __restrict__ pb) {
  // graph-captured steps read (lr, grad_scale) from device memory, so a replayed HIP graph
  // follows the LR schedule / loss scale without being re-captured
  if (hyper != nullptr) {
    lr = hyper[0];
    grad_scale = hyper[1];
  }
  const int2 t = tasks[blockIdx.x];
  const int s = segs[t.x];
  const int n = seg_n[s];
  const int64_t off = seg_off[s];
  const float wd = seg_wd[s];
  const int end = min(t.y + SEPB, n);
  const bool vec = (off & 3) == 0;   // entire-model arenas are unpadded: segments may be unaligned
  for (int i0 = t.y + threadIdx.x * 4; i0 < end; i0 += SNT * 4) {
    if (vec && i0 + 3 < end) {
      float4 pp = *reinterpret_cast<const float4*>(p + off + i0);
      float4 gg = *reinterpret_cast<const float4*>(g + off + i0);
      float x[4] = {pp.x, pp.y, pp.z, pp.w};
      float d[4] = {gg.x, gg.y, gg.z, gg.w};
      float b[4] = {0.f, 0.f, 0.f, 0.f};
      float4 bb;
      if (MOM && !FIRST) {
        bb = *reinterpret_cast<const float4*>(buf + off + i0);
        b[0] = bb.x; b[1] = bb.y; b[2] = bb.z; b[3] = bb.w;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
        x[k] = sgd_elem<MOM, NEST, FIRST>(x[k], d[k], b[k], lr, wd, momentum, dampening,
                                          grad_scale);
      *reinterpret_cast<float4*>(p + off + i0) = make_float4(x[0], x[1], x[2], x[3]);
      if (MOM) *reinterpret_cast<float4*>(buf + off + i0) = make_float4(b[0], b[1], b[2], b[3]);
      if (pb != nullptr)
        *reinterpret_cast<uint2*>(pb + off + i0) =
            make_uint2((uint32_t)f2h(x[0]) | ((uint32_t)f2h(x[1]) << 16),
                       (uint32_t)f2h(x[2]) | ((uint32_t)f2h(x[3]) << 16));
    } else {
      for (int k = 0; k < 4 && i0 + k < end; ++k) {
        const int64_t i = off + i0 + k;
        float bv = MOM && !FIRST ? buf[i] : 0.f;
        p[i] = sgd_elem<MOM, NEST, FIRST>(p[i], g[i], bv, lr, wd, momentum, dampening,
                                          grad_scale);
        if (MOM) buf[i] = bv;
        if (pb != nullptr) pb[i] = f2h(p[i]);
      }
    }
  }
}

// Momentum correction (Lin et al. 2018, DGC; parallel/engine.py), the per-bucket prologue of the
// compressor, over the bucket's ARENA segments (one task = 8192 elements of one segment):
//   g' = g + wmul·wd_s·p      weight decay folded into the gradient BEFORE the velocity, as DGC
//                             does (wmul = 1 / grad_scale keeps it in a loss-scaled gradient's units)
//   u  = mc·u + g'            local velocity
//   g  = u                    the compressor (and its error-feedback residual) sees the velocity
// One read of g, u (and p), one write of g and u: it replaces four ATen passes. Products and sums
// are rounded separately (no fma contraction), as the CPU mirror (parallel/engine.py) computes
// them. The masking of the velocity at the coordinates that were sent happens inside the select kernels (compress.hip
// k_small_select / k_write, SelectArgs::mom) or, for the other codecs, in k_mc_mask.
template <bool WD>
__global__ __launch_bounds__(SNT) void k_mc_prep(float* __restrict__ g, float* __restrict__ u,
                                                 const float* __restrict__ p,
                                                 const int64_t* __restrict__ seg_off,
                                                 const int32_t* __restrict__ seg_n,
                                                 const int32_t* __restrict__ segs,
                                                 const int2* __restrict__ tasks,
                                                 const float* __restrict__ seg_wd, float mc,
                                                 float wmul) {
  // Plain * and + under contract(off): __fmul_rn / __fadd_rn are * / + inside the toolchain's
  // header, where contraction stays on, so after inlining u*mc + g still became one fma (a 1-ulp
  // difference from the CPU mirror)
#pragma clang fp contract(off)
  const int2 t = tasks[blockIdx.x];
  const int s = segs[t.x];
  const int n = seg_n[s];
  const int64_t off = seg_off[s];
  const float wd = WD ? seg_wd[s] * wmul : 0.f;
  const int end = min(t.y + SEPB, n);
  const bool vec = (off & 3) == 0;
  for (int i0 = t.y + threadIdx.x * 4; i0 < end; i0 += SNT * 4) {
    if (vec && i0 + 3 < end) {
      float4 gg = *reinterpret_cast<const float4*>(g + off + i0);
      float4 uu = *reinterpret_cast<const float4*>(u + off + i0);
      if (WD && wd != 0.f) {
        const float4 pp = *reinterpret_cast<const float4*>(p + off + i0);
        gg.x = gg.x + pp.x * wd; gg.y = gg.y + pp.y * wd;
        gg.z = gg.z + pp.z * wd; gg.w = gg.w + pp.w * wd;
      }
      uu.x = uu.x * mc + gg.x; uu.y = uu.y * mc + gg.y;
      uu.z = uu.z * mc + gg.z; uu.w = uu.w * mc + gg.w;
      *reinterpret_cast<float4*>(u + off + i0) = uu;
      *reinterpret_cast<float4*>(g + off + i0) = uu;
    } else {
      for (int k = 0; k < 4 && i0 + k < end; ++k) {
        const int64_t i = off + i0 + k;
        float x = g[i];
        if (WD && wd != 0.f) x = x + p[i] * wd;
        const float v = u[i] * mc + x;
        u[i] = v;
        g[i] = v;
      }
    }
  }
}

void mc_prep(float* g, float* u, const float* p, const int64_t* seg_off, const int32_t* seg_n,
             const int32_t* segs, const int2* tasks, int n_tasks, const float* seg_wd, float mc,
             float wmul, hipStream_t st) {
  if (n_tasks == 0) return;
  if (p != nullptr && seg_wd != nullptr)
    hipLaunchKernelGGL((k_mc_prep<true>), dim3(n_tasks), dim3(SNT), 0, st, g, u, p, seg_off,
                       seg_n, segs, tasks, seg_wd, mc, wmul);
  else
    hipLaunchKernelGGL((k_mc_prep<false>), dim3(n_tasks), dim3(SNT), 0, st, g, u, p, seg_off,
                       seg_n, segs, tasks, seg_wd, mc, wmul);
}

// Momentum factor masking for codecs without a selection (quantisers, thresholds on the dense
// wire): u = 0 where the error-feedback residual is 0, i.e. where the value was sent whole.
__global__ __launch_bounds__(SNT) void k_mc_mask(float* __restrict__ u, const float* __restrict__ e,
                                                 int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * SNT * 4;
  for (int64_t i = ((int64_t)blockIdx.x * SNT + threadIdx.x) * 4; i < n; i += stride) {
    if (i + 3 < n) {
      float4 uu = *reinterpret_cast<const float4*>(u + i);
      const float4 ee = *reinterpret_cast<const float4*>(e + i);
      uu.x = ee.x == 0.f ? 0.f : uu.x; uu.y = ee.y == 0.f ? 0.f : uu.y;
      uu.z = ee.z == 0.f ? 0.f : uu.z; uu.w = ee.w == 0.f ? 0.f : uu.w;
      *reinterpret_cast<float4*>(u + i) = uu;
    } else {
      for (int64_t k = i; k < n; ++k) u[k] = e[k] == 0.f ? 0.f : u[k];
    }
  }
}

void mc_mask(float* u, const float* e, int64_t n, hipStream_t st) {
  if (n <= 0) return;
  int64_t blocks = (n + SNT * 4 - 1) / (SNT * 4);
  blocks = blocks > 2048 ? 2048 : blocks;
  hipLaunchKernelGGL(k_mc_mask, dim3((unsigned)blocks), dim3(SNT), 0, st, u, e, n);
}

void sgd_step(const SgdArgs& a, hipStream_t st) {
  if (a.n_tasks == 0) return;
  const bool mom = a.momentum != 0.f;
  const dim3 grid(a.n_tasks), block(SNT);
#define LW_SGD(M, N, F)                                                                        \
  hipLaunchKernelGGL((k_sgd<M, N, F>), grid, block, 0, st, a.p, a.g, a.buf, a.seg_off, a.seg_n, \
                     a.segs, a.tasks, a.seg_wd, a.lr, a.momentum, a.dampening, a.grad_scale, \
                     a.hyper, a.pb)
  if (!mom) LW_SGD(false, false, false);
  else if (a.nesterov) { if (a.first_step) LW_SGD(true, true, true); else LW_SGD(true, true, false); }
  else { if (a.first_step) LW_SGD(true, false, true); else LW_SGD(true, false, false); }
#undef LW_SGD
}

// One lane adds 1 to a device counter with a vector store (the step count the Philox streams and
// the captured select kernels read; bumped in the graph, not by an ATen add).
__global__ void k_step_bump(int64_t* __restrict__ c) {
  if (threadIdx.x == 0) c[0] = c[0] + 1;
}

void step_bump(int64_t* c, hipStream_t st) {
  hipLaunchKernelGGL(k_step_bump, dim3(1), dim3(64), 0, st, c);
}

}  // namespace lw
