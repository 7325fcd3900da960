// CIFAR-10 batch augmentation on the GPU: random crop from the zero-padded image,
// horizontal flip and cutout, gathered straight into the channels_last (NHWC) training batch in
// the compute dtype — one pass per batch. The reference does the same per image on the host
// (CIFAR10/core.py:121-152 Crop / FlipLR / Cutout, Transform.set_random_choices) and then copies
// each batch to the GPU; here the padded dataset stays resident in HBM and only the per-image
// choices (x0, y0, flip, cutout corner) are drawn on the host once per epoch.
#include "common.h"
#include "lw_kernels.h"
#include "elem16.h"

namespace lw {

// One thread per output element in NHWC order (c fastest): stores are fully coalesced; the
// NCHW source reads hop between C planes of one padded image (L2-resident, 3 x 40 x 40 fp32).
template <bool BF16>
__global__ __launch_bounds__(256) void k_cifar_augment(const float* __restrict__ data,
                                                       const int64_t* __restrict__ idx,
                                                       const int32_t* __restrict__ prm,
                                                       void* __restrict__ out, int B, int C,
                                                       int Hp, int Wp, int crop, int cutout,
                                                       int64_t offset, int Co) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)B * crop * crop * Co;
  if (t >= total) return;
  const int c = (int)(t % Co);
  int64_t r = t / Co;
  if (c >= C) {                               // the zero channels of a padded (Co = 4) batch
    if (BF16) static_cast<uint16_t*>(out)[t] = 0;
    else static_cast<float*>(out)[t] = 0.f;
    return;
  }
  const int x = (int)(r % crop);
  r /= crop;
  const int y = (int)(r % crop);
  const int b = (int)(r / crop);
  // per-image choices of this epoch, row `offset + b` of an [n][5] table
  const int64_t e = offset + b;
  const int32_t* p = prm + 5 * e;             // per-image record [x0, y0, flip, cx, cy]
  const int x0 = p[0], y0 = p[1], flip = p[2], cx = p[3], cy = p[4];
  const int xs = flip ? crop - 1 - x : x;
  float v = data[((idx[b] * C + c) * Hp + (y0 + y)) * Wp + (x0 + xs)];
  if (cutout > 0 && y >= cy && y < cy + cutout && x >= cx && x < cx + cutout) v = 0.f;
  if (BF16) static_cast<uint16_t*>(out)[t] = f2h(v);
  else static_cast<float*>(out)[t] = v;
}

// Co >= C output channels: the ones past C are written as zeros (a 4-channel stem input for the
// MFMA image convolution, ops/conv.py _c4_input, built here instead of by a cast, a fill and a copy)
void cifar_augment(const float* data, const int64_t* idx, const int32_t* prm, void* out, int B,
                   int C, int Hp, int Wp, int crop, int cutout, int64_t offset, bool bf16,
                   hipStream_t st, int Co) {
  if (Co < C) Co = C;
  const int64_t total = (int64_t)B * crop * crop * Co;
  if (total == 0) return;
  const dim3 grid((unsigned)((total + 255) / 256)), block(256);
  if (bf16)
    hipLaunchKernelGGL(k_cifar_augment<true>, grid, block, 0, st, data, idx, prm, out, B, C, Hp,
                       Wp, crop, cutout, offset, Co);
  else
    hipLaunchKernelGGL(k_cifar_augment<false>, grid, block, 0, st, data, idx, prm, out, B, C, Hp,
                       Wp, crop, cutout, offset, Co);
}

}  // namespace lw
