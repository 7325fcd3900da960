// Shared device helpers for the gfx950 (CDNA4, wave64) kernels of layer_wise_aaai20_amd.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace lw {

constexpr int WAVE = 64;

// ---------------------------------------------------------------------------------------------
// Philox4x32-10 counter-based RNG. Bit-identical to layer_wise_aaai20_amd/utils/philox.py so the
// CPU (gloo) path and the GPU path pick the same Random-K masks and dither noise.
// ---------------------------------------------------------------------------------------------
struct u4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u4 philox4x32_10(u4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
    const uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
    c = u4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ uint32_t pick(const u4& v, int j) {
  return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
}

// uniform in [0,1) with 24 random bits (exactly representable in fp32)
__device__ __forceinline__ float u01(uint32_t w) { return (float)(w >> 8) * (1.0f / 16777216.0f); }

// ---------------------------------------------------------------------------------------------
// Block-wide scans / reductions for NT threads (NT multiple of 64). `scratch` needs NT/64 words.
// ---------------------------------------------------------------------------------------------
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* scratch, uint32_t& total) {
  const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < WAVE; o <<= 1) {
    uint32_t y = __shfl_up(x, o, WAVE);
    if (lane >= o) x += y;
  }
  if (lane == WAVE - 1) scratch[w] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NT / WAVE; ++i) {
    const uint32_t t = scratch[i];
    pre += (i < w) ? t : 0u;
    tot += t;
  }
  total = tot;
  __syncthreads();
  return pre + x - v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = WAVE / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, WAVE));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = WAVE / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
  return v;
}

template <int NT>
__device__ __forceinline__ float block_max(float v, float* scratch) {
  v = wave_max(v);
  if ((threadIdx.x & (WAVE - 1)) == 0) scratch[threadIdx.x / WAVE] = v;
  __syncthreads();
  float r = scratch[0];
#pragma unroll
  for (int i = 1; i < NT / WAVE; ++i) r = fmaxf(r, scratch[i]);
  __syncthreads();
  return r;
}

template <int NT>
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  if ((threadIdx.x & (WAVE - 1)) == 0) scratch[threadIdx.x / WAVE] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / WAVE; ++i) r += scratch[i];   // fixed order: deterministic
  __syncthreads();
  return r;
}

}  // namespace lw
