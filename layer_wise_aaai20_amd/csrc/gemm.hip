// bf16 MFMA GEMM for gfx950 with fused prologues / epilogues.
//
//   C[M,N] = pro(A)·pro(B) (+ bias[n]) (ReLU)       bf16 or fp32 output, fp32 accumulation
//
// A(m,k) is read either K-contiguous (A[m*lda+k], "A row-major") or M-contiguous (A[k*lda+m]);
// B(k,n) either K-contiguous (B[n*ldb+k], i.e. an nn.Linear / 1x1-conv weight [N][K]) or
// N-contiguous (B[k*ldb+n]). The four combinations cover forward (x·Wᵀ), data-gradient (dy·W) and
// weight-gradient (dyᵀ·x) of Linear layers and NHWC 1x1 convolutions without any transpose copy:
// K-contiguous tiles are read with ds_read_b128, M/N-contiguous tiles with the gfx950 transposing
// LDS read ds_read_b64_tr_b16 (cdna_hip_programming.md §5.5 T10).
//
// Geometry: 256-thread workgroup = 4 waves as 2x2; the output tile BMxBN is one of 128x128,
// 256x64 (skinny N: 1x1 convs with 64 output channels) or 64x256 (skinny M); BK = 32 or 64 per
// LDS stage; v_mfma_f32_16x16x32_bf16; register-staged double-buffered LDS; workgroup → tile map is
// XCD-aware (the 8 XCDs each get one contiguous run of tiles, so tiles sharing an A row-panel share
// an L2). The epilogue stages the fp32 tile through LDS in two halves for 16-byte coalesced stores.
//
// Fusions (what makes this more than a library GEMM):
//  * prologue PRO_A: a = relu(a*scale[k] + shift[k]) on K-contiguous A — a BatchNorm-apply+ReLU of
//    the *input* folded into a 1x1 convolution (the normalised activation is never materialised);
//  * prologue PRO_B: the same per-n on N-contiguous B — the weight-gradient of that convolution
//    recomputes the normalised activation on load;
//  * epilogue EPI_STATS: per-column Σv and Σv² of the bf16-rounded output per M-tile, written as
//    one coalesced [2][N] row per M-tile ([tiles_m][2][N]); bn.hip folds the rows (k_colsum) and
//    finalizes — the forward statistics pass of the *next* BatchNorm disappears;
//  * split-K (EPI_PARTIAL) writes fp32 slabs that a second kernel reduces in a fixed order
//    (deterministic) and pushes through the same epilogue.
#include "common.h"
#include "gemm_core.h"

#include <algorithm>
#include <vector>

namespace lw {

void gemm_big(const GemmArgs& g, const GemmK& k, int zs, hipStream_t st);   // gemm_big.hip
void gemm_bigp(const GemmArgs& g, const GemmK& k, hipStream_t st);

// Fixed-order reduction of split-K slabs + epilogue. A workgroup owns OT float4 groups of outputs
// and ZT split lanes (ZT*OT = 256): lane z sums splits z, z+ZT, ... in order, then the ZT lane sums
// are added in lane order through LDS — the same order on every run.
__global__ __launch_bounds__(GT) void k_splitk_reduce(const float* __restrict__ partial, int splits,
                                                      int zt_log2, void* __restrict__ C,
                                                      int64_t ldc, const float* __restrict__ bias,
                                                      int relu, int M, int N, int out_bf16,
                                                      const uint16_t* __restrict__ addend,
                                                      const uint8_t* __restrict__ add_bits,
                                                      int accumulate) {
  __shared__ float4 red[GT];
  const int ZT = 1 << zt_log2, OT = GT >> zt_log2;
  const int z = threadIdx.x / OT, o = threadIdx.x % OT;
  const int64_t total = (int64_t)M * N;
  const int64_t i0 = ((int64_t)blockIdx.x * OT + o) * 4;
  const bool vec = (N & 3) == 0;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i0 < total) {
    if (vec) {
#pragma unroll 8
      for (int zz = z; zz < splits; zz += ZT) {
        const float4 v = *reinterpret_cast<const float4*>(partial + (int64_t)zz * total + i0);
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
    } else {
      float t[4] = {0.f, 0.f, 0.f, 0.f};
      for (int zz = z; zz < splits; zz += ZT)
        for (int k = 0; k < 4 && i0 + k < total; ++k) t[k] += partial[(int64_t)zz * total + i0 + k];
      s = make_float4(t[0], t[1], t[2], t[3]);
    }
  }
  red[threadIdx.x] = s;
  __syncthreads();
  if (z != 0 || i0 >= total) return;
  for (int q = 1; q < ZT; ++q) {
    const float4 v = red[q * OT + o];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  float out[4] = {s.x, s.y, s.z, s.w};
  for (int k = 0; k < 4 && i0 + k < total; ++k) {
    const int64_t i = i0 + k;
    const int n = (int)(i % N);
    const int64_t m = i / N;
    float x = out[k];
    if (bias) x += bias[n];
    if (relu) x = fmaxf(x, 0.f);
    if (out_bf16) {
      uint16_t h = f2h(x);
      if (addend)
        h = f2h(h2f(h) + masked_addend1(addend, add_bits, m * ldc + n));
      static_cast<uint16_t*>(C)[m * ldc + n] = h;
    } else {
      float* c = static_cast<float*>(C) + m * ldc + n;
      *c = accumulate ? *c + x : x;
    }
  }
}


// ==========================================================================================
// Streaming GEMM for the large-M / small-K problems of a ResNet bottleneck (the 1x1 convolutions
// of the first two stages: M = N·H·W up to 802816 rows, K = 64..256): HBM-bound, and with one
// output tile per workgroup the tiled kernel above stalls on a full memory latency per tile at
// two workgroups per CU. Here a workgroup is persistent over a strided set of 128-row tiles:
//   * the whole B panel [BN][K] is staged into LDS once and stays resident;
//   * A fragments go straight from HBM into registers in MFMA layout (each lane one 16-byte load
//     per 16x32 fragment: 16 rows x 32 k, full 64-byte row segments) — no LDS round trip — and
//     the NEXT tile's fragments are loaded while the current one runs its MFMAs and epilogue;
//   * the optional BatchNorm-apply+ReLU prologue runs on the A fragments in registers, its
//     per-k coefficients held in LDS;
//   * the epilogue stages the bf16 tile through LDS for 16-byte coalesced stores, adds an
//     optional bf16 addend, and accumulates per-column Σ/Σ² in registers across all of the
//     workgroup's tiles (one statistics row per workgroup, folded by bn.hip k_colsum).
// B is [N][K] (K-contiguous: forward x·Wᵀ) or [K][N] (N-contiguous: data gradient dy·W).
// ==========================================================================================
constexpr int SBM = 128;                        // rows per workgroup tile (4 waves x 32)

template <int K, int BN, bool BKC, bool STATS, bool PRO, bool ADD>
__global__ __launch_bounds__(GT) void k_gemm_stream(const GemmK p) {
  constexpr int LDB = K + 8;                    // B panel row (bf16), 16-B aligned, bank spread
  constexpr int LDO = BN + 8;                   // staged output row (bf16)
  constexpr int KS = K / 32;                    // MFMA k-steps
  constexpr int FN = BN / 16;
  constexpr int B_BYTES = BN * LDB * 2;
  constexpr int C_BYTES = PRO ? 2 * K * 4 : 0;
  constexpr int O_BYTES = SBM * LDO * 2;
  constexpr int F_BYTES = GT * 16 * 4;          // stats fold
  constexpr int TAIL = O_BYTES > F_BYTES ? O_BYTES : F_BYTES;
  __shared__ __attribute__((aligned(16))) uint8_t lds[B_BYTES + C_BYTES + TAIL];
  uint16_t* Bs = reinterpret_cast<uint16_t*>(lds);
  float* coef = reinterpret_cast<float*>(lds + B_BYTES);            // [scale K][shift K]
  uint16_t* Os = reinterpret_cast<uint16_t*>(lds + B_BYTES + C_BYTES);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int n0 = blockIdx.y * BN;

  // ---- stage the B panel (and prologue coefficients) once
  if (BKC) {
    for (int c = threadIdx.x; c < BN * (K / 8); c += GT) {
      const int n = c / (K / 8), k8 = (c % (K / 8)) * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (n0 + n < p.N) v = *reinterpret_cast<const uint4*>(p.B + (int64_t)(n0 + n) * p.ldb + k8);
      *reinterpret_cast<uint4*>(Bs + n * LDB + k8) = v;
    }
  } else {
    for (int c = threadIdx.x; c < K * (BN / 8); c += GT) {
      const int k = c / (BN / 8), n8 = (c % (BN / 8)) * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (n0 + n8 < p.N) v = *reinterpret_cast<const uint4*>(p.B + (int64_t)k * p.ldb + n0 + n8);
      const uint32_t q[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        Bs[(n8 + 2 * j) * LDB + k] = (uint16_t)(q[j] & 0xffffu);
        Bs[(n8 + 2 * j + 1) * LDB + k] = (uint16_t)(q[j] >> 16);
      }
    }
  }
  if (PRO) {
    for (int k = threadIdx.x; k < K; k += GT) {
      coef[k] = p.pro_scale[k];
      coef[K + k] = p.pro_shift[k];
    }
  }
  __syncthreads();

  const int tiles_m = (p.M + SBM - 1) / SBM;
  // A fragments of one tile: [i = 16-row half][s = k-step], 8 bf16 each
  uint4 a_cur[2][KS], a_nxt[2][KS];
  auto load_a = [&](uint4 (&dst)[2][KS], int tm) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = tm * SBM + w * 32 + i * 16 + (l & 15);
      const uint16_t* src = p.A + (int64_t)m * p.lda + 8 * (l >> 4);
#pragma unroll
      for (int s = 0; s < KS; ++s)
        dst[i][s] = m < p.M ? *reinterpret_cast<const uint4*>(src + 32 * s) : make_uint4(0, 0, 0, 0);
    }
  };

  float cs1[8], cs2[8];                         // this thread's 8 columns: Σv, Σv²
#pragma unroll
  for (int k = 0; k < 8; ++k) { cs1[k] = 0.f; cs2[k] = 0.f; }
  const int ccol = (threadIdx.x % (BN / 8)) * 8;  // fixed output column group of this thread
  static_assert(GT % (BN / 8) == 0, "column group must be fixed per thread");

  int tm = blockIdx.x;
  if (tm < tiles_m) load_a(a_cur, tm);
  for (; tm < tiles_m; tm += gridDim.x) {
    const int tn = tm + gridDim.x;
    if (tn < tiles_m) load_a(a_nxt, tn);         // next tile in flight during this one
    if (PRO) {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int kb = 32 * s + 8 * (l >> 4);
        Coef8 co;
#pragma unroll
        for (int j = 0; j < 8; ++j) { co.s[j] = coef[kb + j]; co.t[j] = coef[K + kb + j]; }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int m = tm * SBM + w * 32 + i * 16 + (l & 15);
          if (m < p.M) a_cur[i][s] = affine_relu8(a_cur[i][s], co);
        }
      }
    }
    f32x4 acc[2][FN];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const h16x8 fa0 = __builtin_bit_cast(h16x8, a_cur[0][s]);
      const h16x8 fa1 = __builtin_bit_cast(h16x8, a_cur[1][s]);
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const h16x8 fb = *reinterpret_cast<const h16x8*>(
            Bs + (16 * j + (l & 15)) * LDB + 32 * s + 8 * (l >> 4));
        acc[0][j] = mfma16(fb, fa0, acc[0][j]);
        acc[1][j] = mfma16(fb, fa1, acc[1][j]);
      }
    }
    // ---- epilogue: Cᵀ fragments -> bf16 -> LDS tile -> 16-byte stores
    __syncthreads();                             // previous tile's readback finished
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = w * 32 + i * 16 + (l & 15);
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int c = 16 * j + 4 * (l >> 4);
        const uint32_t lo = (uint32_t)f2h(acc[i][j][0]) | ((uint32_t)f2h(acc[i][j][1]) << 16);
        const uint32_t hi = (uint32_t)f2h(acc[i][j][2]) | ((uint32_t)f2h(acc[i][j][3]) << 16);
        *reinterpret_cast<uint2*>(Os + r * LDO + c) = make_uint2(lo, hi);
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < SBM * (BN / 8); c += GT) {
      const int r = c / (BN / 8);
      const int gm = tm * SBM + r, gn = n0 + ccol;
      if (gm >= p.M || gn >= p.N) continue;
      uint4 v = *reinterpret_cast<const uint4*>(Os + r * LDO + ccol);
      if (STATS) {
        const uint32_t q[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float lo = hlo(q[k]), hi = hhi(q[k]);
          cs1[2 * k] += lo; cs2[2 * k] += lo * lo;
          cs1[2 * k + 1] += hi; cs2[2 * k + 1] += hi * hi;
        }
      }
      uint16_t* dst = static_cast<uint16_t*>(p.C) + (int64_t)gm * p.ldc + gn;
      if (ADD) v = add_h16x8(v, masked_addend8(p.addend, p.add_bits, (int64_t)gm * p.ldc + gn));
      *reinterpret_cast<uint4*>(dst) = v;
    }
    if (tn < tiles_m) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int s = 0; s < KS; ++s) a_cur[i][s] = a_nxt[i][s];
    }
  }
  if (STATS) {
    constexpr int G8 = BN / 8, Q = GT / G8;
    __syncthreads();
    float* fold = reinterpret_cast<float*>(lds + B_BYTES + C_BYTES);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      fold[threadIdx.x * 16 + k] = cs1[k];
      fold[threadIdx.x * 16 + 8 + k] = cs2[k];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < BN; c += GT) {
      const int n = n0 + c;
      if (n >= p.N) continue;
      const int g = c / 8, k = c % 8;
      float a = 0.f, b = 0.f;
      for (int q = 0; q < Q; ++q) {
        a += fold[(q * G8 + g) * 16 + k];
        b += fold[(q * G8 + g) * 16 + 8 + k];
      }
      p.stats[(int64_t)blockIdx.x * 2 * p.N + n] = a;        // [gridDim.x][2][N]
      p.stats[(int64_t)blockIdx.x * 2 * p.N + p.N + n] = b;
    }
  }
}

static bool is_stream_tile(int t) { return t >= GEMM_S64 && t <= GEMM_S256; }
static int stream_bn(int tile) { return tile == GEMM_S64 ? 64 : (tile == GEMM_S128 ? 128 : 256); }

bool gemm_stream_ok(const GemmArgs& g) {
  if (g.tile < GEMM_S64 || g.tile > GEMM_S256) return false;
  const int bn = stream_bn(g.tile);
  const bool kok = g.K == 64 || g.K == 128 || (g.K == 256 && bn <= 128);
  return kok && g.a_kcontig && g.out_bf16 && !g.bias && !g.relu && g.splits <= 1 &&
         !g.accumulate && (g.N % 8) == 0 && (g.ldc % 8) == 0 && (!g.pro_scale || g.pro_on_a) &&
         !(g.pro_scale && !g.b_kcontig) && !(g.addend && g.stats);
}

int gemm_stream_grid_m(const GemmArgs& g) {
  const int panels = (g.N + stream_bn(g.tile) - 1) / stream_bn(g.tile);
  const int tiles = (g.M + SBM - 1) / SBM;
  const int bn = stream_bn(g.tile);               // resident workgroups per CU (LDS-bound)
  int want = 256 * (bn == 64 ? 4 : (bn == 128 ? 2 : 1)) / panels;
  want = want < 1 ? 1 : want;
  return tiles < want ? tiles : want;
}

template <int K, int BN>
static void stream_launch(const GemmArgs& g, const GemmK& k, hipStream_t st) {
  const dim3 grid(gemm_stream_grid_m(g), (g.N + BN - 1) / BN), block(GT);
  const bool stats = g.stats != nullptr, pro = g.pro_scale != nullptr, add = g.addend != nullptr;
  if (g.b_kcontig) {
    if (stats && pro) hipLaunchKernelGGL((k_gemm_stream<K, BN, true, true, true, false>), grid, block, 0, st, k);
    else if (stats) hipLaunchKernelGGL((k_gemm_stream<K, BN, true, true, false, false>), grid, block, 0, st, k);
    else if (add) hipLaunchKernelGGL((k_gemm_stream<K, BN, true, false, false, true>), grid, block, 0, st, k);
    else hipLaunchKernelGGL((k_gemm_stream<K, BN, true, false, false, false>), grid, block, 0, st, k);
  } else {
    if (stats) hipLaunchKernelGGL((k_gemm_stream<K, BN, false, true, false, false>), grid, block, 0, st, k);
    else if (add) hipLaunchKernelGGL((k_gemm_stream<K, BN, false, false, false, true>), grid, block, 0, st, k);
    else hipLaunchKernelGGL((k_gemm_stream<K, BN, false, false, false, false>), grid, block, 0, st, k);
  }
}

static void gemm_stream(const GemmArgs& g, hipStream_t st) {
  GemmK k{g.A, g.B, g.C, nullptr, g.stats, nullptr, g.pro_scale, g.pro_shift, g.addend, g.add_bits, g.lda,
          g.ldb, g.ldc, g.M, g.N, g.K, g.K, 0, 1, 0};
  const int bn = stream_bn(g.tile);
#define LW_SK(KK)                                                                               \
  if (bn == 64) stream_launch<KK, 64>(g, k, st);                                                \
  else if (bn == 128) stream_launch<KK, 128>(g, k, st);                                         \
  else stream_launch<KK, 256>(g, k, st);
  if (g.K == 64) { LW_SK(64) }
  else if (g.K == 128) { LW_SK(128) }
  else { if (bn == 64) stream_launch<256, 64>(g, k, st); else stream_launch<256, 128>(g, k, st); }
#undef LW_SK
}

// ------------------------------------------------------------------------------------------ host
struct TileShape { int bm, bn, bk; };
static bool is_big_tile(int t) {
  return t == GEMM_B256 || t == GEMM_B256x128 || t == GEMM_P256 || t == GEMM_P256x128;
}
static TileShape tile_shape(int t) {
  switch (gemm_base_tile(t)) {
    case GEMM_T128x128x64: return {128, 128, 64};
    case GEMM_T256x64x32: return {256, 64, 32};
    case GEMM_T64x256x32: return {64, 256, 32};
    case GEMM_T256x64x64: return {256, 64, 64};
    case GEMM_T64x64x64: return {64, 64, 64};
    case GEMM_B256: return {256, 256, 64};
    case GEMM_B256x128: return {256, 128, 64};
    case GEMM_P256: return {256, 256, 64};
    case GEMM_P256x128: return {256, 128, 64};
    default: return {128, 128, 32};
  }
}

// rows of C per column-statistics row: the tile height, but 128 for the big tiles (one row per
// wave row, gemm_big.hip)
int stats_rows_bm(int tile) {
  if (is_big_tile(tile)) return 128;
  return tile_shape(tile).bm;
}

int gemm_pick_tile(const GemmArgs& g) {
  if ((g.tile == GEMM_B256 || g.tile == GEMM_B256x128) && !gemm_big_ok(g)) return GEMM_T128x128x64;
  if ((g.tile == GEMM_P256 || g.tile == GEMM_P256x128) && !gemm_bigp_ok(g)) return GEMM_T128x128x64;
  if (g.tile > 0) return g.tile;
  if (g.M <= 64 && g.N <= 64) return GEMM_T64x64x64;
  if (g.N <= 64 && g.M >= 512) return GEMM_T256x64x32;
  if (g.M <= 64 && g.N >= 512) return GEMM_T64x256x32;
  return GEMM_T128x128x32;
}

int gemm_tiles_m(const GemmArgs& g) {
  if (is_stream_tile(g.tile)) return gemm_stream_grid_m(g);   // one statistics row per workgroup
  const int t = gemm_pick_tile(g);
  const int bm = stats_rows_bm(t);
  return (g.M + bm - 1) / bm;
}

static int k_per_split(int K, int splits, int bk) {
  splits = splits < 1 ? 1 : splits;
  int kps = (K + splits - 1) / splits;
  return (kps + bk - 1) / bk * bk;
}

int gemm_splits_used(const GemmArgs& g) {
  if (is_stream_tile(g.tile)) return 1;
  const int pt = gemm_pick_tile(g);
  if (pt == GEMM_P256 || pt == GEMM_P256x128) return 1;
  const int bk = tile_shape(gemm_pick_tile(g)).bk;
  const int kps = k_per_split(g.K, g.splits, bk);
  return (g.K + kps - 1) / kps;
}

template <int BM, int BN, int BK, int EPI, int PRO, int MF>
static void launch_layout(const GemmArgs& g, const GemmK& k, dim3 grid, hipStream_t st) {
  const dim3 block(GT);
#define LW_K(AK, BKC) (k_gemm<BM, BN, BK, AK, BKC, EPI, PRO, CV_NONE, MF>)
  if constexpr (PRO == PRO_A) {
    if (g.b_kcontig) hipLaunchKernelGGL(LW_K(true, true), grid, block, 0, st, k);
    else hipLaunchKernelGGL(LW_K(true, false), grid, block, 0, st, k);
  } else if constexpr (PRO == PRO_B) {
    if (g.a_kcontig) hipLaunchKernelGGL(LW_K(true, false), grid, block, 0, st, k);
    else hipLaunchKernelGGL(LW_K(false, false), grid, block, 0, st, k);
  } else {
    if (g.a_kcontig && g.b_kcontig) hipLaunchKernelGGL(LW_K(true, true), grid, block, 0, st, k);
    else if (g.a_kcontig) hipLaunchKernelGGL(LW_K(true, false), grid, block, 0, st, k);
    else if (g.b_kcontig) hipLaunchKernelGGL(LW_K(false, true), grid, block, 0, st, k);
    else hipLaunchKernelGGL(LW_K(false, false), grid, block, 0, st, k);
  }
#undef LW_K
}

template <int BM, int BN, int BK, int MF>
static void launch_tile(const GemmArgs& g, const GemmK& k, int epi, dim3 grid, hipStream_t st) {
  const int pro = g.pro_scale ? (g.pro_on_a ? PRO_A : PRO_B) : PRO_NONE;
#define LW_E(E)                                                                                  \
  if (pro == PRO_A) launch_layout<BM, BN, BK, E, PRO_A, MF>(g, k, grid, st);                     \
  else if (pro == PRO_B) launch_layout<BM, BN, BK, E, PRO_B, MF>(g, k, grid, st);                \
  else launch_layout<BM, BN, BK, E, PRO_NONE, MF>(g, k, grid, st);
  if (epi == EPI_PARTIAL) { LW_E(EPI_PARTIAL) }
  else if (epi == EPI_STATS) { LW_E(EPI_STATS) }
  else { LW_E(EPI_STORE) }
#undef LW_E
}

// ------------------------------------------------------------------------------------------
// Deferred split-K reduces. Inside a splitk_defer(true) scope (ops/block.py: a bottleneck's
// weight gradients accumulated straight into the gradient arena) a split GEMM / conv leaves its
// fp32 slabs for splitk_flush, which the gradient engine calls before it reads the arena
// (parallel/engine.py): one launch reduces every pending slab set — ResNet-50 ran 54 reduce
// launches a step, at ~5 µs of launch floor each in the replayed graph. Per element the sum is
// k_splitk_reduce's, same split lanes and fold order, so the result is identical.
// ------------------------------------------------------------------------------------------
struct ReduceJob {
  const float* partial;
  float* C;
  int64_t ldc, blk_lo;       // output row stride; first block of this job in the launch
  int splits, zl, M, N, accumulate;
};
constexpr int kMaxReduceJobs = 24;
struct ReduceJobs {
  ReduceJob j[kMaxReduceJobs];
  int n;
};

__global__ __launch_bounds__(GT) void k_splitk_reduce_multi(const ReduceJobs jobs) {
  __shared__ float4 red[GT];
  int ji = 0;
  for (int q = 1; q < jobs.n; ++q)
    if ((int64_t)blockIdx.x >= jobs.j[q].blk_lo) ji = q;
  const ReduceJob J = jobs.j[ji];
  const int ZT = 1 << J.zl, OT = GT >> J.zl;
  const int z = threadIdx.x / OT, o = threadIdx.x % OT;
  const int64_t total = (int64_t)J.M * J.N;
  const int64_t i0 = (((int64_t)blockIdx.x - J.blk_lo) * OT + o) * 4;
  const bool vec = (J.N & 3) == 0;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i0 < total) {
    if (vec) {
#pragma unroll 8
      for (int zz = z; zz < J.splits; zz += ZT) {
        const float4 v = *reinterpret_cast<const float4*>(J.partial + (int64_t)zz * total + i0);
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
    } else {
      float t[4] = {0.f, 0.f, 0.f, 0.f};
      for (int zz = z; zz < J.splits; zz += ZT)
        for (int k = 0; k < 4 && i0 + k < total; ++k) t[k] += J.partial[(int64_t)zz * total + i0 + k];
      s = make_float4(t[0], t[1], t[2], t[3]);
    }
  }
  red[threadIdx.x] = s;
  __syncthreads();
  if (z != 0 || i0 >= total) return;
  for (int q = 1; q < ZT; ++q) {
    const float4 v = red[q * OT + o];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  const float out[4] = {s.x, s.y, s.z, s.w};
  for (int k = 0; k < 4 && i0 + k < total; ++k) {
    const int64_t i = i0 + k;
    float* c = J.C + (i / J.N) * J.ldc + (int)(i % J.N);
    *c = J.accumulate ? *c + out[k] : out[k];
  }
}

static bool g_defer = false, g_last_deferred = false;
static std::vector<ReduceJob> g_pending;

void splitk_set_defer(bool on) { g_defer = on; }
bool splitk_take_deferred() {
  const bool r = g_last_deferred;
  g_last_deferred = false;
  return r;
}

static int splitk_lanes(int zs) {
  int zl = 0;                                    // split lanes: up to 32, no more than splits
  while (zl < 5 && (2 << zl) <= zs) ++zl;
  return zl;
}

int splitk_flush(hipStream_t st) {
  const int n = (int)g_pending.size();
  for (int b = 0; b < n; b += kMaxReduceJobs) {
    ReduceJobs jobs{};
    jobs.n = std::min(kMaxReduceJobs, n - b);
    int64_t blocks = 0;
    for (int q = 0; q < jobs.n; ++q) {
      ReduceJob r = g_pending[b + q];
      const int64_t groups = ((int64_t)r.M * r.N + 3) / 4, ot = GT >> r.zl;
      r.blk_lo = blocks;
      blocks += (groups + ot - 1) / ot;
      jobs.j[q] = r;
    }
    hipLaunchKernelGGL(k_splitk_reduce_multi, dim3((unsigned)blocks), dim3(GT), 0, st, jobs);
  }
  g_pending.clear();
  return n;
}

// Drop every queued reduce without launching anything (a step that failed between a deferred
// GEMM and the flush — a capture that fell back to eager, a backward that raised): the slabs it
// names were never (or only partly) written, and reducing them into the arena would add garbage.
int splitk_discard() {
  const int n = (int)g_pending.size();
  g_pending.clear();
  g_defer = false;
  g_last_deferred = false;
  return n;
}

int splitk_pending() { return (int)g_pending.size(); }

void splitk_reduce(const GemmArgs& g, int zs, hipStream_t st) {
  if (g_defer && !g.out_bf16 && g.bias == nullptr && !g.relu && g.addend == nullptr) {
    g_pending.push_back(ReduceJob{g.partial, static_cast<float*>(g.C), g.ldc, 0, zs,
                                  splitk_lanes(zs), g.M, g.N, g.accumulate ? 1 : 0});
    g_last_deferred = true;
    return;
  }
  const int64_t total = (int64_t)g.M * g.N;
  const int zl = splitk_lanes(zs);
  const int64_t groups = (total + 3) / 4, ot = GT >> zl;
  const dim3 rg((unsigned)((groups + ot - 1) / ot));
  hipLaunchKernelGGL(k_splitk_reduce, rg, dim3(GT), 0, st, g.partial, zs, zl, g.C, g.ldc, g.bias,
                     g.relu, g.M, g.N, g.out_bf16 ? 1 : 0, g.addend, g.add_bits,
                     g.accumulate ? 1 : 0);
}

void gemm_tile_shape(int t, int& bm, int& bn, int& bk) {
  const TileShape ts = tile_shape(t);
  bm = ts.bm; bn = ts.bn; bk = ts.bk;
}

int gemm_k_per_split(int K, int splits, int bk) { return k_per_split(K, splits, bk); }

void gemm_bf16(const GemmArgs& g, hipStream_t st) {
  if (is_stream_tile(g.tile)) {
    gemm_stream(g, st);
    return;
  }
  const int t = gemm_pick_tile(g);
  const TileShape ts = tile_shape(t);
  const bool persist = t == GEMM_P256 || t == GEMM_P256x128;     // never split
  const int kps = persist ? g.K : k_per_split(g.K, g.splits, ts.bk);
  const int zs = (g.K + kps - 1) / kps;
  const int tiles = ((g.M + ts.bm - 1) / ts.bm) * ((g.N + ts.bn - 1) / ts.bn);
  const int epi = zs > 1 ? EPI_PARTIAL
                          : (g.stats ? (g.bst_x ? EPI_BSTATS : EPI_STATS) : EPI_STORE);
  GemmK k{g.A, g.B, g.C, g.partial, g.stats, zs > 1 ? nullptr : g.bias, g.pro_scale, g.pro_shift,
          g.addend, g.add_bits, g.lda, g.ldb, g.ldc, g.M, g.N, g.K, kps, zs > 1 ? 0 : g.relu,
          g.out_bf16 ? 1 : 0, g.accumulate ? 1 : 0};
  k.a_bytes = g.a_bytes;
  k.b_bytes = g.b_bytes;
  k.bst_x = g.bst_x;
  k.bst_mean = g.bst_mean;
  k.bst_scale = g.bst_scale;
  k.bst_shift = g.bst_shift;
  k.bst_bits = g.bst_bits;
  const dim3 grid(tiles, zs);
  if (persist) {
    gemm_bigp(g, k, st);
    return;
  }
  if (t == GEMM_B256 || t == GEMM_B256x128) {
    gemm_big(g, k, zs, st);
    if (zs > 1) splitk_reduce(g, zs, st);
    return;
  }
  if (gemm_is_mf32(t)) {
    switch (gemm_base_tile(t)) {
      case GEMM_T128x128x64: launch_tile<128, 128, 64, 32>(g, k, epi, grid, st); break;
      case GEMM_T256x64x32: launch_tile<256, 64, 32, 32>(g, k, epi, grid, st); break;
      case GEMM_T64x256x32: launch_tile<64, 256, 32, 32>(g, k, epi, grid, st); break;
      case GEMM_T256x64x64: launch_tile<256, 64, 64, 32>(g, k, epi, grid, st); break;
      case GEMM_T64x64x64: launch_tile<64, 64, 64, 32>(g, k, epi, grid, st); break;
      default: launch_tile<128, 128, 32, 32>(g, k, epi, grid, st); break;
    }
  } else {
    switch (t) {
      case GEMM_T128x128x64: launch_tile<128, 128, 64, 16>(g, k, epi, grid, st); break;
      case GEMM_T256x64x32: launch_tile<256, 64, 32, 16>(g, k, epi, grid, st); break;
      case GEMM_T64x256x32: launch_tile<64, 256, 32, 16>(g, k, epi, grid, st); break;
      case GEMM_T256x64x64: launch_tile<256, 64, 64, 16>(g, k, epi, grid, st); break;
      case GEMM_T64x64x64: launch_tile<64, 64, 64, 16>(g, k, epi, grid, st); break;
      default: launch_tile<128, 128, 32, 16>(g, k, epi, grid, st); break;
    }
  }
  if (zs > 1) splitk_reduce(g, zs, st);
}

}  // namespace lw
