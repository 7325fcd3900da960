// One element of the fused SGD update (torch.optim.SGD semantics: grad unscale, weight decay,
// momentum with dampening, Nesterov), shared by the arena-wide k_sgd (optim.hip) and the
// decode-and-step k_unpack_sgd (compress.hip) so that both round identically: every product and
// sum is rounded on its own (no fma contraction), as the CPU path of optim/flat_sgd.py computes.
#pragma once

namespace lw {

template <bool MOM, bool NEST, bool FIRST>
__device__ __forceinline__ float sgd_elem(float x, float g, float& b, float lr, float wd,
                                          float momentum, float dampening, float grad_scale) {
#pragma clang fp contract(off)
  float dp = g * grad_scale;
  if (wd != 0.f) dp = dp + wd * x;
  if (MOM) {
    b = FIRST ? dp : momentum * b + (1.f - dampening) * dp;
    dp = NEST ? dp + momentum * b : b;
  }
  return x - lr * dp;
}

}  // namespace lw
