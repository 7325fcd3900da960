// bf16 MFMA GEMM for gfx950 with fused epilogues.
//
//   C[M,N] = A·B (+ bias[n]) (ReLU)            bf16 or fp32 output, fp32 accumulation
//
// A(m,k) is read either K-contiguous (A[m*lda+k], "A row-major") or M-contiguous (A[k*lda+m]);
// B(k,n) either K-contiguous (B[n*ldb+k], i.e. an nn.Linear / 1x1-conv weight [N][K]) or
// N-contiguous (B[k*ldb+n]). The four combinations cover forward (x·Wᵀ), data-gradient (dy·W) and
// weight-gradient (dyᵀ·x) of Linear layers and NHWC 1x1 convolutions without any transpose copy:
// K-contiguous tiles are read with ds_read_b128, M/N-contiguous tiles with the gfx950 transposing
// LDS read ds_read_b64_tr_b16 (cdna_hip_programming.md §5.5 T10).
//
// Geometry: 128x128 output tile per 256-thread workgroup (4 waves as 2x2, 64x64 per wave),
// BK = 32, v_mfma_f32_16x16x32_bf16 (4x4 per wave per k-step), register-staged double-buffered
// LDS, LDS-staged coalesced epilogue. Split-K (grid.z) writes fp32 partial slabs that a second
// kernel reduces in a fixed order (deterministic) and pushes through the same epilogue.
#include "common.h"
#include "lw_kernels.h"

namespace lw {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int GT = 256;
constexpr int TM = 128, TN = 128, TK = 32;
constexpr int KPAD = 8;              // bf16 elements of padding per LDS row
constexpr int LDK = TK + KPAD;       // K-contiguous tile row (40 el = 80 B)
constexpr int LDMN = TM + KPAD;      // M/N-contiguous tile row (136 el = 272 B)

template <bool KC> struct TileCfg;
template <> struct TileCfg<true> { static constexpr int ELEMS = TM * LDK; };
template <> struct TileCfg<false> { static constexpr int ELEMS = TK * LDMN; };

__device__ __forceinline__ uint16_t bf16_rne(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)((u >> 16) | ((u & 0xffff) ? 0x40 : 0));
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// Global -> registers: two 16-byte chunks per thread for a 128x32 (or 32x128) bf16 tile.
// KC: rows = 128 (m or n), 4 chunks of 8 k each. !KC: rows = 32 (k), 16 chunks of 8 m/n each.
template <bool KC>
__device__ __forceinline__ void load_tile(const uint16_t* __restrict__ P, int64_t ld, int row0,
                                          int rows_total, int k0, int K, uint4 r[2]) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = threadIdx.x + h * GT;
    int rr, cc;     // tile-local row / 8-element chunk
    bool ok;
    int64_t off;
    if (KC) {
      rr = c >> 2; cc = c & 3;
      const int gr = row0 + rr, gk = k0 + cc * 8;
      ok = gr < rows_total && gk < K;
      off = (int64_t)gr * ld + gk;
    } else {
      rr = c >> 4; cc = c & 15;
      const int gk = k0 + rr, gr = row0 + cc * 8;
      ok = gk < K && gr < rows_total;
      off = (int64_t)gk * ld + gr;
    }
    r[h] = ok ? *reinterpret_cast<const uint4*>(P + off) : make_uint4(0, 0, 0, 0);
  }
}

template <bool KC>
__device__ __forceinline__ void store_tile(uint16_t* __restrict__ S, const uint4 r[2]) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = threadIdx.x + h * GT;
    uint16_t* d = KC ? S + (c >> 2) * LDK + (c & 3) * 8 : S + (c >> 4) * LDMN + (c & 15) * 8;
    *reinterpret_cast<uint4*>(d) = r[h];
  }
}

// MFMA operand fragment (8 bf16 along k) for tile row/col `i` (0..127) and k-group g = lane>>4.
template <bool KC>
__device__ __forceinline__ bf16x8 load_frag(const uint16_t* S, int i_base) {
  const int l = threadIdx.x & 63;
  if (KC) {
    const uint16_t* p = S + (i_base + (l & 15)) * LDK + 8 * (l >> 4);
    return *reinterpret_cast<const bf16x8*>(p);
  } else {
    const int g = l >> 4, t = l & 15, q = t >> 2, p4 = t & 3;
    typedef __attribute__((address_space(3))) i16x4 lds_v4;
    const uint16_t* p0 = S + (8 * g + q) * LDMN + i_base + 4 * p4;
    const uint16_t* p1 = p0 + 4 * LDMN;
    const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(p0));
    const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(p1));
    typedef short i16x8 __attribute__((ext_vector_type(8)));
    const i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

template <bool OUT_BF16>
__device__ __forceinline__ void store_out8(void* C, int64_t off, const float v[8]) {
  if (OUT_BF16) {
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = (uint32_t)bf16_rne(v[2 * k]) | ((uint32_t)bf16_rne(v[2 * k + 1]) << 16);
    *reinterpret_cast<uint4*>(static_cast<uint16_t*>(C) + off) = make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    float* c = static_cast<float*>(C) + off;
    reinterpret_cast<float4*>(c)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(c)[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
}

// Epilogue on a 128x128 fp32 tile staged in LDS: bias, ReLU, conversion, 16-B coalesced stores.
template <bool OUT_BF16>
__device__ __forceinline__ void epilogue_store(const float* Cs, int ldcs, void* C, int64_t ldc,
                                               int m0, int n0, int M, int N,
                                               const float* __restrict__ bias, bool relu) {
  // 128 rows x 16 chunks of 8 columns
  for (int c = threadIdx.x; c < TM * (TN / 8); c += GT) {
    const int r = c >> 4, cc = (c & 15) * 8;
    const int gm = m0 + r, gn = n0 + cc;
    if (gm >= M || gn >= N) continue;
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float x = Cs[r * ldcs + cc + k];
      if (bias) x += (gn + k < N) ? bias[gn + k] : 0.f;
      if (relu) x = fmaxf(x, 0.f);
      v[k] = x;
    }
    if (gn + 8 <= N) {
      store_out8<OUT_BF16>(C, (int64_t)gm * ldc + gn, v);
    } else {
      for (int k = 0; k < 8 && gn + k < N; ++k) {
        if (OUT_BF16) static_cast<uint16_t*>(C)[(int64_t)gm * ldc + gn + k] = bf16_rne(v[k]);
        else static_cast<float*>(C)[(int64_t)gm * ldc + gn + k] = v[k];
      }
    }
  }
}

template <bool AKC, bool BKC, bool OUT_BF16>
__global__ __launch_bounds__(GT) void k_gemm(const uint16_t* __restrict__ A, int64_t lda,
                                             const uint16_t* __restrict__ B, int64_t ldb,
                                             void* __restrict__ C, int64_t ldc,
                                             float* __restrict__ partial,   // split-K slabs
                                             const float* __restrict__ bias, int relu, int M,
                                             int N, int K, int k_per_split) {
  constexpr int AE = TileCfg<AKC>::ELEMS, BE = TileCfg<BKC>::ELEMS;
  constexpr int STAGE = AE + BE;
  constexpr int CS_FLOATS = TM * (TN + 4);
  constexpr int LDS_BYTES_STAGES = 2 * STAGE * 2;
  constexpr int LDS_BYTES = LDS_BYTES_STAGES > CS_FLOATS * 4 ? LDS_BYTES_STAGES : CS_FLOATS * 4;
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
  uint16_t* st = reinterpret_cast<uint16_t*>(lds);

  const int n0 = blockIdx.x * TN, m0 = blockIdx.y * TM;
  const int kbeg = blockIdx.z * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int wr = w >> 1, wc = w & 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[2], rb[2];
  int cur = 0;
  if (kbeg < kend) {
    load_tile<AKC>(A, lda, m0, M, kbeg, kend, ra);
    load_tile<BKC>(B, ldb, n0, N, kbeg, kend, rb);
    store_tile<AKC>(st, ra);
    store_tile<BKC>(st + AE, rb);
  }
  __syncthreads();
  for (int k0 = kbeg; k0 < kend; k0 += TK) {
    const bool more = k0 + TK < kend;
    if (more) {
      load_tile<AKC>(A, lda, m0, M, k0 + TK, kend, ra);
      load_tile<BKC>(B, ldb, n0, N, k0 + TK, kend, rb);
    }
    const uint16_t* As = st + cur * STAGE;
    const uint16_t* Bs = As + AE;
    bf16x8 fa[4], fb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = load_frag<AKC>(As, wr * 64 + i * 16);
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = load_frag<BKC>(Bs, wc * 64 + j * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    if (more) {
      uint16_t* nx = st + (cur ^ 1) * STAGE;
      store_tile<AKC>(nx, ra);
      store_tile<BKC>(nx + AE, rb);
    }
    __syncthreads();
    cur ^= 1;
  }

  // stage the fp32 tile in LDS (C/D map: col = lane&15, row = 4*(lane>>4) + r)
  float* Cs = reinterpret_cast<float*>(lds);
  constexpr int LDC = TN + 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Cs[(wr * 64 + i * 16 + 4 * (l >> 4) + r) * LDC + wc * 64 + j * 16 + (l & 15)] = acc[i][j][r];
  __syncthreads();
  if (gridDim.z > 1) {
    float* P = partial + (int64_t)blockIdx.z * M * N;
    for (int c = threadIdx.x; c < TM * (TN / 4); c += GT) {
      const int r = c >> 5, cc = (c & 31) * 4;
      const int gm = m0 + r, gn = n0 + cc;
      if (gm >= M || gn >= N) continue;
      if (gn + 4 <= N && (N & 3) == 0) {
        *reinterpret_cast<float4*>(P + (int64_t)gm * N + gn) =
            make_float4(Cs[r * LDC + cc], Cs[r * LDC + cc + 1], Cs[r * LDC + cc + 2], Cs[r * LDC + cc + 3]);
      } else {
        for (int k = 0; k < 4 && gn + k < N; ++k) P[(int64_t)gm * N + gn + k] = Cs[r * LDC + cc + k];
      }
    }
    return;
  }
  epilogue_store<OUT_BF16>(Cs, LDC, C, ldc, m0, n0, M, N, bias, relu != 0);
}

// Fixed-order reduction of split-K slabs + epilogue.
template <bool OUT_BF16>
__global__ __launch_bounds__(GT) void k_splitk_reduce(const float* __restrict__ partial, int splits,
                                                      void* __restrict__ C, int64_t ldc,
                                                      const float* __restrict__ bias, int relu,
                                                      int M, int N) {
  const int64_t i = ((int64_t)blockIdx.x * GT + threadIdx.x);
  const int64_t total = (int64_t)M * N;
  if (i >= total) return;
  float s = 0.f;
  for (int z = 0; z < splits; ++z) s += partial[(int64_t)z * total + i];
  const int n = (int)(i % N);
  const int m = (int)(i / N);
  if (bias) s += bias[n];
  if (relu) s = fmaxf(s, 0.f);
  if (OUT_BF16) static_cast<uint16_t*>(C)[(int64_t)m * ldc + n] = bf16_rne(s);
  else static_cast<float*>(C)[(int64_t)m * ldc + n] = s;
}

void gemm_bf16(const GemmArgs& g, hipStream_t st) {
  const int splits = g.splits < 1 ? 1 : g.splits;
  int kps = (g.K + splits - 1) / splits;
  kps = (kps + TK - 1) / TK * TK;
  const int zs = (g.K + kps - 1) / kps;
  dim3 grid((g.N + TN - 1) / TN, (g.M + TM - 1) / TM, zs);
  dim3 block(GT);
#define LW_G(AK, BK, OB)                                                                       \
  hipLaunchKernelGGL((k_gemm<AK, BK, OB>), grid, block, 0, st, g.A, g.lda, g.B, g.ldb, g.C,      \
                     g.ldc, g.partial, zs > 1 ? nullptr : g.bias, zs > 1 ? 0 : g.relu, g.M, g.N, \
                     g.K, kps)
#define LW_G2(OB)                                                                              \
  if (g.a_kcontig && g.b_kcontig) LW_G(true, true, OB);                                       \
  else if (g.a_kcontig) LW_G(true, false, OB);                                                \
  else if (g.b_kcontig) LW_G(false, true, OB);                                                \
  else LW_G(false, false, OB);
  if (g.out_bf16) { LW_G2(true) } else { LW_G2(false) }
#undef LW_G2
#undef LW_G
  if (zs > 1) {
    const int64_t total = (int64_t)g.M * g.N;
    const dim3 rg((unsigned)((total + GT - 1) / GT));
    if (g.out_bf16)
      hipLaunchKernelGGL(k_splitk_reduce<true>, rg, block, 0, st, g.partial, zs, g.C, g.ldc, g.bias, g.relu, g.M, g.N);
    else
      hipLaunchKernelGGL(k_splitk_reduce<false>, rg, block, 0, st, g.partial, zs, g.C, g.ldc, g.bias, g.relu, g.M, g.N);
  }
}

int gemm_splits_used(int K, int splits) {
  splits = splits < 1 ? 1 : splits;
  int kps = (K + splits - 1) / splits;
  kps = (kps + TK - 1) / TK * TK;
  return (K + kps - 1) / kps;
}

}  // namespace lw
