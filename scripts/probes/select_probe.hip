// Standalone timing probe of the fused Top-K select chain (csrc/compress.hip) on one
// entire-model segment — the shape of BASELINE config 3 (CIFAR AlexNet, ~9 M gradients, K = 1 %,
// error feedback). Built with different -D knobs (LW_HIST_CP, LW_HIST_TPB_MIN, ...) into separate
// binaries so variants can be compared on one box without rebuilding the extension:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I layer_wise_aaai20_amd/csrc [-D...] \
//     scripts/probes/select_probe.hip -o /tmp/select_probe
//   select_probe [N] [K fraction] [iters] [mc] [g.f32 e.f32]
// Prints one JSON line: mean µs of the chain (events around select_compress only; the gradient
// and residual are restored from pristine copies before every call).
#include "compress.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(2);                                                                  \
    }                                                                                \
  } while (0)

__device__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

// normal(0, 1) x a per-64k-block scale in [1e-3, 1]: layers of very different gradient scales
__global__ void k_fill(float* p, int64_t n, uint32_t salt, float mul) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float u1 = ((hash32((uint32_t)i * 2u + salt) >> 8) + 1) * (1.f / 16777217.f);
  const float u2 = (hash32((uint32_t)i * 2u + 1u + salt) >> 8) * (1.f / 16777216.f);
  const float z = sqrtf(-2.f * logf(u1)) * cosf(6.2831853f * u2);
  const float lvl = (hash32((uint32_t)(i >> 16) + 77u) >> 8) * (1.f / 16777216.f);
  p[i] = z * mul * powf(10.f, -3.f * lvl);
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? std::atoll(argv[1]) : 9042734;
  const double kf = argc > 2 ? std::atof(argv[2]) : 0.01;
  const int iters = argc > 3 ? std::atoi(argv[3]) : 50;
  const bool mc = argc > 4 && std::atoi(argv[4]) != 0;   // fused momentum correction (u, p, wd)
  const int m = (int)std::max<int64_t>(1, (int64_t)(kf * (double)n));
  const int cap = m + std::max(64, m / 64);
  const int ntasks = (int)((n + lw::kLargeEPB - 1) / lw::kLargeEPB);

  float *g0, *e0, *g, *e;
  CK(hipMalloc(&g0, n * 4)); CK(hipMalloc(&e0, n * 4));
  CK(hipMalloc(&g, n * 4)); CK(hipMalloc(&e, n * 4));
  const int fb = (int)((n + 255) / 256);
  hipLaunchKernelGGL(k_fill, dim3(fb), dim3(256), 0, 0, g0, n, 1u, 1.f);
  hipLaunchKernelGGL(k_fill, dim3(fb), dim3(256), 0, 0, e0, n, 99u, 0.3f);
  if (argc > 6) {                        // real gradient / residual (scripts/probes/dump_em_grad.py)
    for (int w = 0; w < 2; ++w) {
      std::vector<float> h(n);
      FILE* f = std::fopen(argv[5 + w], "rb");
      if (f == nullptr || std::fread(h.data(), 4, n, f) != (size_t)n) {
        std::fprintf(stderr, "cannot read %lld floats from %s\n", (long long)n, argv[5 + w]);
        return 2;
      }
      std::fclose(f);
      CK(hipMemcpy(w == 0 ? g0 : e0, h.data(), 4 * n, hipMemcpyHostToDevice));
    }
  }

  std::vector<int64_t> seg_off = {0, n}, cap_off = {0, cap};
  std::vector<int32_t> seg_n = {(int32_t)n}, keep = {m}, large = {0}, task_lo = {0, ntasks};
  std::vector<int2> tasks(ntasks);
  for (int t = 0; t < ntasks; ++t) tasks[t] = make_int2(0, t * lw::kLargeEPB);
  auto up = [](const void* h, size_t bytes) {
    void* d;
    CK(hipMalloc(&d, bytes));
    CK(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice));
    return d;
  };
  lw::SelectArgs a{};
  a.g = g; a.ef = e;
  a.seg_off = (const int64_t*)up(seg_off.data(), 16);
  a.seg_n = (const int32_t*)up(seg_n.data(), 4);
  a.keep = (const int32_t*)up(keep.data(), 4);
  a.cap_off = (const int64_t*)up(cap_off.data(), 16);
  a.large_segs = (const int32_t*)up(large.data(), 4);
  a.tasks = (const int2*)up(tasks.data(), sizeof(int2) * ntasks);
  a.task_lo = (const int32_t*)up(task_lo.data(), 8);
  a.n_small = 0; a.n_large = 1; a.n_tasks = ntasks; a.max_seg_tasks = ntasks;
  CK(hipMalloc(&a.hist, 4 * lw::HIST_WORDS));
  CK(hipMemset(a.hist, 0, 4 * lw::HIST_WORDS));
  CK(hipMalloc(&a.st_large, sizeof(lw::SelState)));
  CK(hipMalloc(&a.cnt, sizeof(uint2) * ntasks * lw::kWriteSub));
  CK(hipMalloc(&a.pre, sizeof(uint2) * ntasks * lw::kWriteSub));
  CK(hipMalloc(&a.pairs, sizeof(int2) * cap));
  unsigned long long* ovf;
  CK(hipMalloc(&ovf, 8));
  CK(hipMemset(ovf, 0, 8));
  a.overflow = ovf;

  if (mc) {                              // u = 0.9·u + g + 1e-4·p in the first pass
    float *u, *p, *wd;
    CK(hipMalloc(&u, n * 4)); CK(hipMalloc(&p, n * 4)); CK(hipMalloc(&wd, 4));
    hipLaunchKernelGGL(k_fill, dim3(fb), dim3(256), 0, 0, u, n, 7u, 0.1f);
    hipLaunchKernelGGL(k_fill, dim3(fb), dim3(256), 0, 0, p, n, 11u, 1.f);
    const float w = 1e-4f;
    CK(hipMemcpy(wd, &w, 4, hipMemcpyHostToDevice));
    a.mcx = lw::McArgs{u, p, wd, 0.9f, 1.f};
  }
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t ea, eb;
  CK(hipEventCreate(&ea)); CK(hipEventCreate(&eb));
  double tot = 0.0;
  for (int it = 0; it < iters + 10; ++it) {
    CK(hipMemcpyAsync(g, g0, n * 4, hipMemcpyDeviceToDevice, st));
    CK(hipMemcpyAsync(e, e0, n * 4, hipMemcpyDeviceToDevice, st));
    CK(hipEventRecord(ea, st));
    lw::select_compress(a, lw::KM_TOPK, lw::OUT_PAIRS, true, st, false);
    CK(hipEventRecord(eb, st));
    CK(hipEventSynchronize(eb));
    float ms;
    CK(hipEventElapsedTime(&ms, ea, eb));
    if (it >= 10) tot += ms;
  }
  // one more call from the pristine inputs: FNV hashes of the payload and the residual, so runs
  // of different builds (-D knobs) can be compared bit for bit
  CK(hipMemcpyAsync(g, g0, n * 4, hipMemcpyDeviceToDevice, st));
  CK(hipMemcpyAsync(e, e0, n * 4, hipMemcpyDeviceToDevice, st));
  lw::select_compress(a, lw::KM_TOPK, lw::OUT_PAIRS, true, st, false);
  CK(hipStreamSynchronize(st));
  std::vector<int2> hp(cap);
  std::vector<float> he(n), hg(n);
  CK(hipMemcpy(hp.data(), a.pairs, sizeof(int2) * cap, hipMemcpyDeviceToHost));
  CK(hipMemcpy(he.data(), e, 4 * n, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hg.data(), g, 4 * n, hipMemcpyDeviceToHost));
  auto fnv = [](const void* p, size_t bytes) {
    uint64_t x = 1469598103934665603ull;
    const unsigned char* c = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < bytes; ++i) { x ^= c[i]; x *= 1099511628211ull; }
    return (unsigned long long)x;
  };
  std::vector<uint32_t> hh(lw::HIST_WORDS);
  CK(hipMemcpy(hh.data(), a.hist, 4 * lw::HIST_WORDS, hipMemcpyDeviceToHost));
  uint64_t hsum = 0;
  for (uint32_t x : hh) hsum += x;
  std::printf("{\"pairs_hash\": %llu, \"e_hash\": %llu, \"g_hash\": %llu, "
              "\"hist_left\": %llu}\n", fnv(hp.data(), sizeof(int2) * cap), fnv(he.data(), 4 * n),
              fnv(hg.data(), 4 * n), (unsigned long long)hsum);
  lw::SelState s;
  CK(hipMemcpy(&s, a.st_large, sizeof(s), hipMemcpyDeviceToHost));
  unsigned long long o;
  CK(hipMemcpy(&o, ovf, 8, hipMemcpyDeviceToHost));
  std::printf("{\"n\": %lld, \"keep\": %d, \"tasks\": %d, \"chain_us\": %.2f, \"sent\": %u, "
              "\"tkey\": %u, \"overflow\": %llu, \"cp\": %d, \"tpb_min\": %d, \"split_max\": %d}\n",
              (long long)n, m, ntasks, 1000.0 * tot / iters, s.total, s.tkey, o, LW_HIST_CP,
              LW_HIST_TPB_MIN, LW_HIST_SPLIT_MAX);
  return 0;
}
