// Grid sweeps of the remaining streaming passes of the ResNet-50 step (bs 256) that do not run at
// the HBM rate: the downsample block's dual BN backward (reduce + apply, layer-1 shape
// M = 802816, C = 256) and the stem's pool forward / backward (N = 256, 112x112 -> 56x56, C = 64).
// HIP events over buffers beyond the 256 MiB Infinity Cache.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I layer_wise_aaai20_amd/csrc \
//     scripts/probes/bn_stream_probe2.hip -o build/probe/bn_stream_probe2
#include "bn.hip"
#include <cstdio>
#include <vector>

using namespace lw;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

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

static void rep(const char* name, float us, double mb) {
  printf("%-52s %8.1f us  %7.1f MB  %6.2f TB/s\n", name, us, mb, mb / us);
}

static void geom(int64_t M, int C, int target, int64_t& rpb, int& nb) {
  const int nsl = reduce_slices(C);
  const int G = C / nsl / 8, R = BNT / G;
  const int64_t rb = (target + nsl - 1) / nsl;
  rpb = (M + rb - 1) / rb;
  rpb = (rpb + R - 1) / R * R;
  nb = (int)((M + rpb - 1) / rpb);
}

int main() {
  Timer T;
  {  // dual BN backward, layer 1
    const int64_t M = 802816;
    const int C = 256;
    const int64_t n = M * C, n8 = n / 8;
    uint16_t *x, *x2, *dy, *dx, *dx2;
    uint8_t* bits;
    float *mu, *A, *part, *part2;
    CK(hipMalloc(&x, n * 2)); CK(hipMalloc(&x2, n * 2)); CK(hipMalloc(&dy, n * 2));
    CK(hipMalloc(&dx, n * 2)); CK(hipMalloc(&dx2, n * 2)); CK(hipMalloc(&bits, n8));
    CK(hipMalloc(&mu, C * 4)); CK(hipMalloc(&A, C * 4));
    CK(hipMalloc(&part, 2 * C * 8192 * 4)); CK(hipMalloc(&part2, 2 * C * 8192 * 4));
    CK(hipMemset(x, 0x3f, n * 2)); CK(hipMemset(x2, 0x3e, n * 2)); CK(hipMemset(dy, 0x3d, n * 2));
    CK(hipMemset(bits, 0x5a, n8)); CK(hipMemset(mu, 0, C * 4)); CK(hipMemset(A, 0, C * 4));
    const double MB = (double)n * 2 / 1e6;
    for (int target : {256, 512, 768, 1024}) {
      int64_t rpb;
      int nb;
      geom(M, C, target, rpb, nb);
      char nm[80];
      snprintf(nm, 80, "dual reduce, %d row blocks x %d slices", nb, reduce_slices(C));
      rep(nm, T.run([&] {
        hipLaunchKernelGGL((k_bn_reduce<uint16_t, 1, 3, 4, true>), dim3(nb, reduce_slices(C)), dim3(BNT), 0, 0,
                           x, dy, (const uint16_t*)nullptr, bits, mu, (const float*)nullptr,
                           (const float*)nullptr, M, C, rpb, part, x2, mu, part2); }), 3 * MB + n8 / 1e6);
    }
    for (int g : {512, 768, 1024, 1536, 2048, 4096}) {
      char nm[80];
      snprintf(nm, 80, "dual bwd apply, grid %d", g);
      rep(nm, T.run([&] {
        hipLaunchKernelGGL(k_bn_bwd_apply_dual, dim3(g), dim3(BNT), 0, 0, x, x2, dy, bits, A, A, A,
                           A, A, A, dx, dx2, n8, C); }), 5 * MB + n8 / 1e6);
    }
    for (void* p : {(void*)x, (void*)x2, (void*)dy, (void*)dx, (void*)dx2, (void*)bits, (void*)mu,
                    (void*)A, (void*)part, (void*)part2}) CK(hipFree(p));
  }
  {  // stem pool, 112x112 -> 56x56
    const int N = 256, H = 112, W = 112, C = 64, Ho = 56, Wo = 56;
    const int64_t nin = (int64_t)N * H * W * C, nout = (int64_t)N * Ho * Wo * C;
    uint16_t *x, *out, *dp, *dx;
    uint8_t* idx;
    float *sc, *part, *A;
    CK(hipMalloc(&x, nin * 2)); CK(hipMalloc(&dx, nin * 2)); CK(hipMalloc(&out, nout * 2));
    CK(hipMalloc(&dp, nout * 2)); CK(hipMalloc(&idx, nout)); CK(hipMalloc(&sc, C * 4));
    CK(hipMalloc(&part, 2 * C * 8192 * 4)); CK(hipMalloc(&A, C * 4));
    CK(hipMemset(x, 0x3f, nin * 2)); CK(hipMemset(dp, 0x3d, nout * 2)); CK(hipMemset(idx, 4, nout));
    std::vector<float> one(C, 1.f);
    CK(hipMemcpy(sc, one.data(), C * 4, hipMemcpyHostToDevice));
    CK(hipMemset(A, 0, C * 4));
    const PoolGeom g{N, H, W, C, Ho, Wo, 3, 2, 1};
    const double inMB = nin * 2 / 1e6, outMB = nout * 2 / 1e6;
    const int64_t total = (int64_t)N * Ho * Wo * (C / 8);
    rep("stem pool fwd (shipped, one output per thread)", T.run([&] {
      hipLaunchKernelGGL(k_stem_pool_fwd, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, 0,
                         x, sc, sc, out, idx, g); }), inMB + outMB + nout / 1e6);
    const int64_t P = (int64_t)N * Ho * Wo;
    for (int target : {256, 512, 1024, 2048, 4096}) {
      int64_t rpb;
      int nb;
      geom(P, C, target, rpb, nb);
      char nm[80];
      snprintf(nm, 80, "stem pool bwd_s2 apply, %d blocks", nb);
      rep(nm, T.run([&] {
        hipLaunchKernelGGL((k_stem_pool_bwd_s2<1>), dim3(nb), dim3(BNT), 0, 0, dp, idx, x, sc, sc, sc,
                           A, A, A, dx, (float*)nullptr, g, rpb); }), 2 * inMB + outMB + nout / 1e6);
      snprintf(nm, 80, "stem pool reduce_out, %d blocks", nb);
      rep(nm, T.run([&] {
        hipLaunchKernelGGL(k_stem_pool_reduce_out, dim3(nb), dim3(BNT), 0, 0, dp, out, idx, x, sc,
                           sc, sc, sc, part, g, rpb); }), 2 * outMB + nout / 1e6);
    }
    for (void* p : {(void*)x, (void*)dx, (void*)out, (void*)dp, (void*)idx, (void*)sc, (void*)part,
                    (void*)A}) CK(hipFree(p));
  }
  return 0;
}
