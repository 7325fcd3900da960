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
      for (int k = 0; k < 4; ++k) {
        float dp = d[k] * grad_scale;
        if (wd != 0.f) dp = dp + wd * x[k];
        if (MOM) {
          b[k] = FIRST ? dp : momentum * b[k] + (1.f - dampening) * dp;
          dp = NEST ? dp + momentum * b[k] : b[k];
        }
        x[k] = x[k] - lr * dp;
      }
      *reinterpret_cast<float4*>(p + off + i0) = make_float4(x[0], x[1], x[2], x[3]);
      if (MOM) *reinterpret_cast<float4*>(buf + off + i0) = make_float4(b[0], b[1], b[2], b[3]);
      if (pb != nullptr)
        *reinterpret_cast<uint2*>(pb + off + i0) =
            make_uint2((uint32_t)f2h(x[0]) | ((uint32_t)f2h(x[1]) << 16),
                       (uint32_t)f2h(x[2]) | ((uint32_t)f2h(x[3]) << 16));
    } else {
      for (int k = 0; k < 4 && i0 + k < end; ++k) {
        const int64_t i = off + i0 + k;
        float x = p[i];
        float dp = g[i] * grad_scale;
        if (wd != 0.f) dp = dp + wd * x;
        if (MOM) {
          const float bv = FIRST ? dp : momentum * buf[i] + (1.f - dampening) * dp;
          buf[i] = bv;
          dp = NEST ? dp + momentum * bv : bv;
        }
        p[i] = x - lr * dp;
        if (pb != nullptr) pb[i] = f2h(p[i]);
      }
    }
  }
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

}  // namespace lw
