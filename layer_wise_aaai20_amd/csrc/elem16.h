// The 16-bit element of the fused path: activations, gradients, weight mirrors and MFMA operands.
//
// Storage is raw 16-bit words (uint16_t) everywhere; only the conversions and the matrix-core
// instruction depend on the format. The default build is bf16. The lwaaai16 build (csrc/build.py
// PRECISIONS, compiled with -DLW_FP16) is the same kernels for IEEE fp16 — the reference's --fp16
// recipe (IMAGENET/training/train_imagenet_nv.py:410-428, fp16util.py:21-138) on the MFMA path:
// v_mfma_f32_16x16x32_f16 / _32x32x16_f16 instead of _bf16, fp32 accumulation and fp32 epilogue
// math in both.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace lw {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct ElemBF16 {
  typedef __bf16 V8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ float f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
  static __device__ __forceinline__ float lo(uint32_t w) { return __uint_as_float(w << 16); }
  static __device__ __forceinline__ float hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
  // round to nearest even: a plain cast, lowered to the gfx950 v_cvt_pk_bf16_f32 (NaN stays NaN)
  static __device__ __forceinline__ uint16_t rne(float x) {
    return __builtin_bit_cast(uint16_t, static_cast<__bf16>(x));
  }
  static __device__ __forceinline__ f32x4 mfma(V8 a, V8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ f32x16 mfma32(V8 a, V8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};

struct ElemF16 {
  typedef _Float16 V8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ float f(uint16_t h) {
    return (float)__builtin_bit_cast(_Float16, h);
  }
  static __device__ __forceinline__ float lo(uint32_t w) { return f((uint16_t)(w & 0xffffu)); }
  static __device__ __forceinline__ float hi(uint32_t w) { return f((uint16_t)(w >> 16)); }
  // v_cvt_f16_f32: round to nearest even, overflow to ±inf (the static loss scale keeps the
  // gradients in range, as in the reference's fp16 recipe)
  static __device__ __forceinline__ uint16_t rne(float x) {
    return __builtin_bit_cast(uint16_t, static_cast<_Float16>(x));
  }
  static __device__ __forceinline__ f32x4 mfma(V8 a, V8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ f32x16 mfma32(V8 a, V8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};

#ifdef LW_FP16
using E16 = ElemF16;
#else
using E16 = ElemBF16;
#endif

typedef E16::V8 h16x8;

__device__ __forceinline__ float h2f(uint16_t h) { return E16::f(h); }
__device__ __forceinline__ float hlo(uint32_t w) { return E16::lo(w); }     // element 0 of a word
__device__ __forceinline__ float hhi(uint32_t w) { return E16::hi(w); }     // element 1 of a word
__device__ __forceinline__ uint16_t f2h(float x) { return E16::rne(x); }
__device__ __forceinline__ float h_round(float x) { return E16::f(E16::rne(x)); }
__device__ __forceinline__ uint32_t pack2h(float a, float b) {
  return (uint32_t)f2h(a) | ((uint32_t)f2h(b) << 16);
}
__device__ __forceinline__ f32x4 mfma16(h16x8 a, h16x8 b, f32x4 c) { return E16::mfma(a, b, c); }
// v_mfma_f32_32x32x16_{bf16,f16}: lane l holds A[row l&31][k = 8(l>>5) + j] and B[k][col l&31]
// (j = 0..7); result register r of lane l is D[row (r&3) + 8(r>>2) + 4(l>>5)][col l&31]
__device__ __forceinline__ f32x16 mfma32(h16x8 a, h16x8 b, f32x16 c) { return E16::mfma32(a, b, c); }

}  // namespace lw
