// Streaming-efficiency probe for the BatchNorm passes at the ResNet-50 layer-1 shapes (bs 256):
// M = 802816 rows, C = 256 (BN3) / 64 (BN1, BN2), bf16 NHWC. Times the shipped kernels of
// csrc/bn.hip against variants and against plain copy kernels of the same byte mix, with HIP
// events over buffers larger than the 256 MiB Infinity Cache (so the numbers are HBM rates).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I layer_wise_aaai20_amd/csrc \
//     scripts/probes/bn_stream_probe.hip -o build/probe/bn_stream_probe
#include "bn.hip"
#include <cstdio>
#include <vector>

using namespace lw;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

// reference streams: copy (1R1W), 2R1W, 2R0W
__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ a, uint4* __restrict__ o, int64_t n) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) o[i] = a[i];
}
__global__ __launch_bounds__(256) void k_add2(const uint4* __restrict__ a, const uint4* __restrict__ b,
                                              uint4* __restrict__ o, int64_t n) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    uint4 x = a[i], y = b[i];
    o[i] = make_uint4(x.x ^ y.x, x.y ^ y.y, x.z ^ y.z, x.w ^ y.w);
  }
}
__global__ __launch_bounds__(256) void k_sum2(const uint4* __restrict__ a, const uint4* __restrict__ b,
                                              uint32_t* __restrict__ o, int64_t n) {
  uint32_t s = 0;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    uint4 x = a[i], y = b[i];
    s += x.x ^ y.x ^ x.w ^ y.w;
  }
  if (s == 0x12345) o[0] = s;
}

// forward apply variant: U grid-strides per iteration, every load issued first; NT stores
template <int U, bool NTS, bool BITS>
__global__ __launch_bounds__(256) void k_apply_v(const uint16_t* __restrict__ x, const uint16_t* __restrict__ res,
                                                 uint16_t* __restrict__ y, const float* __restrict__ scale,
                                                 const float* __restrict__ shift, uint8_t* __restrict__ bits_out,
                                                 int64_t n8, int C) {
  const int G = C / 8;
  const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t step = (int64_t)gridDim.x * 256;
  const int c0 = (int)(t0 % G) * 8;
  float sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { sc[k] = scale[c0 + k]; sh[k] = shift[c0 + k]; }
  for (int64_t i = t0; i < n8; i += U * step) {
    uint4 vx[U], vr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = i + u * step;
      if (j < n8) {
        vx[u] = *reinterpret_cast<const uint4*>(x + j * 8);
        vr[u] = *reinterpret_cast<const uint4*>(res + j * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = i + u * step;
      if (j >= n8) break;
      float v[8], r[8];
      V8<uint16_t>::cvt(vx[u], v);
      V8<uint16_t>::cvt(vr[u], r);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = fmaxf(fmaf(v[k], sc[k], sh[k]) + r[k], 0.f);
      uint32_t w[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) w[k] = (uint32_t)f2h(v[2 * k]) | ((uint32_t)f2h(v[2 * k + 1]) << 16);
      uint4* yp = reinterpret_cast<uint4*>(y + j * 8);
      typedef uint32_t v4u __attribute__((ext_vector_type(4)));
      if (NTS) __builtin_nontemporal_store(v4u{w[0], w[1], w[2], w[3]}, reinterpret_cast<v4u*>(yp));
      else *yp = make_uint4(w[0], w[1], w[2], w[3]);
      if (BITS) {
        uint32_t b = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) b |= (h2f(f2h(v[k])) > 0.f ? 1u : 0u) << k;
        if (NTS) __builtin_nontemporal_store((uint8_t)b, bits_out + j);
        else bits_out[j] = (uint8_t)b;
      }
    }
  }
}

// backward apply variant (mask from the bitmap): U grid-strides in flight
template <int U, bool NTS>
__global__ __launch_bounds__(256) void k_bwd_apply_v(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy,
                                                     const uint8_t* __restrict__ bits, const float* __restrict__ A,
                                                     const float* __restrict__ B, const float* __restrict__ Cc,
                                                     uint16_t* __restrict__ dx, int64_t n8, int C) {
  const int G = C / 8;
  const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t step = (int64_t)gridDim.x * 256;
  const int c0 = (int)(t0 % G) * 8;
  float ca[8], cb[8], cc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { ca[k] = A[c0 + k]; cb[k] = B[c0 + k]; cc[k] = Cc[c0 + k]; }
  for (int64_t i = t0; i < n8; i += U * step) {
    uint4 vx[U], vd[U];
    uint32_t vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = i + u * step;
      if (j < n8) {
        vx[u] = *reinterpret_cast<const uint4*>(x + j * 8);
        vd[u] = *reinterpret_cast<const uint4*>(dy + j * 8);
        vb[u] = bits[j];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = i + u * step;
      if (j >= n8) break;
      float xv[8], d[8], o[8];
      V8<uint16_t>::cvt(vx[u], xv);
      V8<uint16_t>::cvt(vd[u], d);
      mask_bits(d, vb[u]);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = ca[k] * d[k] + cb[k] * xv[k] + cc[k];
      uint32_t w[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) w[k] = (uint32_t)f2h(o[2 * k]) | ((uint32_t)f2h(o[2 * k + 1]) << 16);
      uint4* p = reinterpret_cast<uint4*>(dx + j * 8);
      typedef uint32_t v4u __attribute__((ext_vector_type(4)));
      if (NTS) __builtin_nontemporal_store(v4u{w[0], w[1], w[2], w[3]}, reinterpret_cast<v4u*>(p));
      else *p = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

struct Timer {
  hipEvent_t a, b;
  Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
  template <class F> float run(F f, int iters = 10) {
    for (int i = 0; i < 2; ++i) f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.f / iters;
  }
};

int main(int argc, char** argv) {
  const int64_t M = 802816;
  Timer T;
  for (int C : {256, 64}) {
    const int64_t n = M * C, n8 = n / 8;
    uint16_t *x, *r, *y, *dy, *dx;
    uint8_t* bits;
    float *sc, *sh, *A, *B, *Cc, *part;
    CK(hipMalloc(&x, n * 2)); CK(hipMalloc(&r, n * 2)); CK(hipMalloc(&y, n * 2));
    CK(hipMalloc(&dy, n * 2)); CK(hipMalloc(&dx, n * 2)); CK(hipMalloc(&bits, n8));
    CK(hipMalloc(&sc, C * 4)); CK(hipMalloc(&sh, C * 4)); CK(hipMalloc(&A, C * 4));
    CK(hipMalloc(&B, C * 4)); CK(hipMalloc(&Cc, C * 4)); CK(hipMalloc(&part, 2 * C * 8192 * 4));
    CK(hipMemset(x, 0x3f, n * 2)); CK(hipMemset(r, 0x3e, n * 2)); CK(hipMemset(dy, 0x3d, n * 2));
    CK(hipMemset(bits, 0x5a, n8));
    std::vector<float> one(C, 1.f);
    for (float* p : {sc, A, B, Cc}) CK(hipMemcpy(p, one.data(), C * 4, hipMemcpyHostToDevice));
    CK(hipMemset(sh, 0, C * 4));
    uint32_t* sink;
    CK(hipMalloc(&sink, 4));
    const double MB = (double)n * 2 / 1e6;
    auto rep = [&](const char* name, float us, double mb) {
      printf("C=%4d %-44s %8.1f us  %7.1f MB  %6.2f TB/s\n", C, name, us, mb, mb / us);
    };
    const int64_t nv = n / 8;   // uint4 count
    for (int g : {256, 512, 1024, 2048}) {
      char nm[64];
      snprintf(nm, 64, "copy 1R1W grid %d", g);
      rep(nm, T.run([&] { hipLaunchKernelGGL(k_copy, dim3(g), dim3(256), 0, 0, (const uint4*)x, (uint4*)y, nv); }), 2 * MB);
      snprintf(nm, 64, "xor 2R1W grid %d", g);
      rep(nm, T.run([&] { hipLaunchKernelGGL(k_add2, dim3(g), dim3(256), 0, 0, (const uint4*)x, (const uint4*)r, (uint4*)y, nv); }), 3 * MB);
      snprintf(nm, 64, "sum 2R grid %d", g);
      rep(nm, T.run([&] { hipLaunchKernelGGL(k_sum2, dim3(g), dim3(256), 0, 0, (const uint4*)x, (const uint4*)r, sink, nv); }), 2 * MB);
    }
    const int ag = apply_grid(n8, C, 4096);   // (the round-5 grid)
    const double fb = 3 * MB + n8 / 1e6;
    rep("k_bn_apply<1,relu> + bits (shipped)", T.run([&] {
      hipLaunchKernelGGL((k_bn_apply<uint16_t, 1, true>), dim3(ag), dim3(BNT), 0, 0, x, r, y, sc, sh,
                         (const float*)nullptr, (const float*)nullptr, bits, n8, C); }), fb);
    for (int g : {256, 512, 768, 1024, 1536}) {
      char nm[64];
      snprintf(nm, 64, "k_bn_apply<1,relu>+bits grid %d", g);
      rep(nm, T.run([&] {
        hipLaunchKernelGGL((k_bn_apply<uint16_t, 1, true>), dim3(g), dim3(BNT), 0, 0, x, r, y, sc, sh,
                           (const float*)nullptr, (const float*)nullptr, bits, n8, C); }), fb);
      snprintf(nm, 64, "k_bn_bwd_apply<3> grid %d", g);
      rep(nm, T.run([&] {
        hipLaunchKernelGGL((k_bn_bwd_apply<uint16_t, 3, false>), dim3(g), dim3(BNT), 0, 0, x, dy,
                           (const uint16_t*)nullptr, bits, sc, sh, sc, sh, sh, dx, (uint16_t*)nullptr, n8, C); }),
          3 * MB + n8 / 1e6);
      snprintf(nm, 64, "k_bn_apply<0,relu> grid %d", g);
      rep(nm, T.run([&] {
        hipLaunchKernelGGL((k_bn_apply<uint16_t, 0, true>), dim3(g), dim3(BNT), 0, 0, x, r, y, sc, sh,
                           (const float*)nullptr, (const float*)nullptr, (uint8_t*)nullptr, n8, C); }), 2 * MB);
      snprintf(nm, 64, "apply_v U2 bits grid %d", g);
      rep(nm, T.run([&] { hipLaunchKernelGGL((k_apply_v<2, false, true>), dim3(g), dim3(256), 0, 0, x, r, y, sc, sh, bits, n8, C); }), fb);
    }
    for (int target : {128, 256, 384}) {
      const int nsl = reduce_slices(C);
      const int Gs = C / nsl / 8, R = BNT / Gs;
      const int64_t rbk = (target + nsl - 1) / nsl;
      int64_t rp = (M + rbk - 1) / rbk;
      rp = (rp + R - 1) / R * R;
      const int nbk = (int)((M + rp - 1) / rp);
      char nm[64];
      snprintf(nm, 64, "k_bn_reduce<1,3,U4> %d blocks", nbk * nsl);
      rep(nm, T.run([&] {
        hipLaunchKernelGGL((k_bn_reduce<uint16_t, 1, 3, 4>), dim3(nbk, nsl), dim3(BNT), 0, 0, x, dy,
                           (const uint16_t*)nullptr, bits, sc, (const float*)nullptr, (const float*)nullptr, M, C, rp,
                           part, (const uint16_t*)nullptr, (const float*)nullptr, (float*)nullptr); }), 2 * MB + n8 / 1e6);
    }
    rep("k_bn_apply<1,relu> no bits", T.run([&] {
      hipLaunchKernelGGL((k_bn_apply<uint16_t, 1, true>), dim3(ag), dim3(BNT), 0, 0, x, r, y, sc, sh,
                         (const float*)nullptr, (const float*)nullptr, (uint8_t*)nullptr, n8, C); }), 3 * MB);
    for (int g : {2048, 4096, 8192}) {
      const int gg = (g + (ag % g)) ;  // (grid multiple of G/gcd: 4096-based grids already are)
      (void)gg;
      char nm[64];
      snprintf(nm, 64, "apply_v U2 bits grid %d", g);
      rep(nm, T.run([&] { hipLaunchKernelGGL((k_apply_v<2, false, true>), dim3(g), dim3(256), 0, 0, x, r, y, sc, sh, bits, n8, C); }), fb);
      snprintf(nm, 64, "apply_v U4 bits grid %d", g);
      rep(nm, T.run([&] { hipLaunchKernelGGL((k_apply_v<4, false, true>), dim3(g), dim3(256), 0, 0, x, r, y, sc, sh, bits, n8, C); }), fb);
      snprintf(nm, 64, "apply_v U4 bits NT grid %d", g);
      rep(nm, T.run([&] { hipLaunchKernelGGL((k_apply_v<4, true, true>), dim3(g), dim3(256), 0, 0, x, r, y, sc, sh, bits, n8, C); }), fb);
      snprintf(nm, 64, "apply_v U4 nobits grid %d", g);
      rep(nm, T.run([&] { hipLaunchKernelGGL((k_apply_v<4, false, false>), dim3(g), dim3(256), 0, 0, x, r, y, sc, sh, bits, n8, C); }), 3 * MB);
    }
    // backward
    int64_t rpb;
    int nb;
    reduce_geometry(M, C, rpb, nb);
    const double rb = 2 * MB + n8 / 1e6;
    rep("k_bn_reduce<1,3,U4> (shipped)", T.run([&] {
      hipLaunchKernelGGL((k_bn_reduce<uint16_t, 1, 3, 4>), dim3(nb, reduce_slices(C)), dim3(BNT), 0, 0, x, dy,
                         (const uint16_t*)nullptr, bits, sc, (const float*)nullptr, (const float*)nullptr, M, C, rpb,
                         part, (const uint16_t*)nullptr, (const float*)nullptr, (float*)nullptr); }), rb);
    rep("k_bn_reduce<1,3,U8>", T.run([&] {
      hipLaunchKernelGGL((k_bn_reduce<uint16_t, 1, 3, 8>), dim3(nb, reduce_slices(C)), dim3(BNT), 0, 0, x, dy,
                         (const uint16_t*)nullptr, bits, sc, (const float*)nullptr, (const float*)nullptr, M, C, rpb,
                         part, (const uint16_t*)nullptr, (const float*)nullptr, (float*)nullptr); }), rb);
    for (int target : {1024, 2048, 4096}) {
      const int nsl = reduce_slices(C);
      const int Gs = C / nsl / 8, R = BNT / Gs;
      const int64_t rbk = (target + nsl - 1) / nsl;
      int64_t rp = (M + rbk - 1) / rbk;
      rp = (rp + R - 1) / R * R;
      const int nbk = (int)((M + rp - 1) / rp);
      char nm[64];
      snprintf(nm, 64, "k_bn_reduce<1,3,U4> %d blocks", nbk * nsl);
      rep(nm, T.run([&] {
        hipLaunchKernelGGL((k_bn_reduce<uint16_t, 1, 3, 4>), dim3(nbk, nsl), dim3(BNT), 0, 0, x, dy,
                           (const uint16_t*)nullptr, bits, sc, (const float*)nullptr, (const float*)nullptr, M, C, rp,
                           part, (const uint16_t*)nullptr, (const float*)nullptr, (float*)nullptr); }), rb);
    }
    const double ab = 3 * MB + n8 / 1e6;
    rep("k_bn_bwd_apply<3> (shipped)", T.run([&] {
      hipLaunchKernelGGL((k_bn_bwd_apply<uint16_t, 3, false>), dim3(ag), dim3(BNT), 0, 0, x, dy,
                         (const uint16_t*)nullptr, bits, sc, sh, A, B, Cc, dx, (uint16_t*)nullptr, n8, C); }), ab);
    for (int g : {2048, 4096, 8192}) {
      char nm[64];
      snprintf(nm, 64, "bwd_apply_v U2 grid %d", g);
      rep(nm, T.run([&] { hipLaunchKernelGGL((k_bwd_apply_v<2, false>), dim3(g), dim3(256), 0, 0, x, dy, bits, A, B, Cc, dx, n8, C); }), ab);
      snprintf(nm, 64, "bwd_apply_v U4 grid %d", g);
      rep(nm, T.run([&] { hipLaunchKernelGGL((k_bwd_apply_v<4, false>), dim3(g), dim3(256), 0, 0, x, dy, bits, A, B, Cc, dx, n8, C); }), ab);
      snprintf(nm, 64, "bwd_apply_v U4 NT grid %d", g);
      rep(nm, T.run([&] { hipLaunchKernelGGL((k_bwd_apply_v<4, true>), dim3(g), dim3(256), 0, 0, x, dy, bits, A, B, Cc, dx, n8, C); }), ab);
    }
    for (void* p : {(void*)x, (void*)r, (void*)y, (void*)dy, (void*)dx, (void*)bits, (void*)sc, (void*)sh,
                    (void*)A, (void*)B, (void*)Cc, (void*)part, (void*)sink})
      CK(hipFree(p));
  }
  return 0;
}
