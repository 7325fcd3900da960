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
#include "lw_kernels.h"

namespace lw {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int GT = 256;
constexpr int PAD = 8;                   // bf16 elements of padding per LDS row
enum { EPI_STORE = 0, EPI_PARTIAL = 1, EPI_STATS = 2 };
enum { PRO_NONE = 0, PRO_A = 1, PRO_B = 2 };

// f32 -> bf16, round to nearest even: a plain cast, which hipcc lowers to the gfx950 hardware
// conversion v_cvt_pk_bf16_f32 (NaN stays NaN), instead of integer bit arithmetic.
__device__ __forceinline__ uint16_t bf16_rne(float f) {
  return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f));
}
__device__ __forceinline__ float bf16_round(float f) { return __uint_as_float((uint32_t)bf16_rne(f) << 16); }

// bf16 + bf16 -> bf16 per element (fp32 add, one rounding): the same arithmetic as a separate
// elementwise add of two bf16 tensors, so fusing the residual-gradient add changes no bits.
__device__ __forceinline__ uint4 add_bf16x8(uint4 a, uint4 b) {
  const uint32_t x[4] = {a.x, a.y, a.z, a.w}, y[4] = {b.x, b.y, b.z, b.w};
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float lo = __uint_as_float(x[k] << 16) + __uint_as_float(y[k] << 16);
    const float hi = __uint_as_float(x[k] & 0xffff0000u) + __uint_as_float(y[k] & 0xffff0000u);
    w[k] = (uint32_t)bf16_rne(lo) | ((uint32_t)bf16_rne(hi) << 16);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// 8 addend values of a chunk, zeroed where the ReLU bitmap (bits of the chunk's first element,
// chunk-aligned) is clear.
__device__ __forceinline__ uint4 masked_addend8(const uint16_t* __restrict__ add,
                                                const uint8_t* __restrict__ bits, int64_t e) {
  uint4 a = *reinterpret_cast<const uint4*>(add + e);
  if (bits) {
    const uint32_t b = bits[e >> 3];
    const uint32_t m0 = ((b & 1u) ? 0xffffu : 0u) | ((b & 2u) ? 0xffff0000u : 0u);
    const uint32_t m1 = ((b & 4u) ? 0xffffu : 0u) | ((b & 8u) ? 0xffff0000u : 0u);
    const uint32_t m2 = ((b & 16u) ? 0xffffu : 0u) | ((b & 32u) ? 0xffff0000u : 0u);
    const uint32_t m3 = ((b & 64u) ? 0xffffu : 0u) | ((b & 128u) ? 0xffff0000u : 0u);
    a = make_uint4(a.x & m0, a.y & m1, a.z & m2, a.w & m3);
  }
  return a;
}

__device__ __forceinline__ float masked_addend1(const uint16_t* __restrict__ add,
                                                const uint8_t* __restrict__ bits, int64_t e) {
  if (bits && !((bits[e >> 3] >> (e & 7)) & 1u)) return 0.f;
  return __uint_as_float((uint32_t)add[e] << 16);
}

// R = extent of the tile along m (A) or n (B). KC tiles are stored [R][BK+PAD], the others
// [BK][R+PAD]; both are moved as 16-byte chunks of 8 contiguous elements.
template <int R, int BK, bool KC> struct Tile {
  static constexpr int LD = KC ? BK + PAD : R + PAD;
  static constexpr int ELEMS = KC ? R * LD : BK * LD;
  static constexpr int CPR = KC ? BK / 8 : R / 8;     // chunks per stored row
  static constexpr int PER_T = R * BK / 8 / GT;       // chunks per thread
  static_assert(R * BK / 8 % GT == 0, "tile must split evenly over the workgroup");
};

template <int R, int BK, bool KC>
__device__ __forceinline__ void chunk_pos(int c, int& rr, int& cc) {
  using T = Tile<R, BK, KC>;
  rr = c / T::CPR;
  cc = c % T::CPR;
}

// Global -> registers. `cont` returns the contiguous-dimension index of each chunk (k for KC,
// m/n otherwise) for the prologue; `ok` marks chunks inside the matrix (others are zero).
template <int R, int BK, bool KC>
__device__ __forceinline__ void load_tile(const uint16_t* __restrict__ P, int64_t ld, int row0,
                                          int rows_total, int k0, int kend,
                                          uint4 (&r)[Tile<R, BK, KC>::PER_T],
                                          int (&cont)[Tile<R, BK, KC>::PER_T], uint32_t& okmask) {
  using T = Tile<R, BK, KC>;
  okmask = 0;
#pragma unroll
  for (int h = 0; h < T::PER_T; ++h) {
    int rr, cc;
    chunk_pos<R, BK, KC>(threadIdx.x + h * GT, rr, cc);
    int64_t off;
    bool ok;
    if (KC) {
      const int gr = row0 + rr, gk = k0 + cc * 8;
      ok = gr < rows_total && gk < kend;
      off = (int64_t)gr * ld + gk;
      cont[h] = gk;
    } else {
      const int gk = k0 + rr, gr = row0 + cc * 8;
      ok = gk < kend && gr < rows_total;
      off = (int64_t)gk * ld + gr;
      cont[h] = gr;
    }
    r[h] = ok ? *reinterpret_cast<const uint4*>(P + off) : make_uint4(0, 0, 0, 0);
    okmask |= (ok ? 1u : 0u) << h;
  }
}

// Prologue coefficients of the 8 channels one thread's chunks cover. Every chunk a thread stages
// has the same contiguous-dimension offset within the tile (the chunks-per-row count divides the
// workgroup size), so one set of 8 scale/shift values serves all of them: per K-step for PRO_A
// (channel = k), once per kernel for PRO_B (channel = n).
struct Coef8 { float s[8], t[8]; };

__device__ __forceinline__ void load_coef8(Coef8& c, const float* __restrict__ sc,
                                           const float* __restrict__ sh, int j, int limit) {
  if (j + 8 <= limit) {
    const float4 s0 = *reinterpret_cast<const float4*>(sc + j);
    const float4 s1 = *reinterpret_cast<const float4*>(sc + j + 4);
    const float4 h0 = *reinterpret_cast<const float4*>(sh + j);
    const float4 h1 = *reinterpret_cast<const float4*>(sh + j + 4);
    c.s[0] = s0.x; c.s[1] = s0.y; c.s[2] = s0.z; c.s[3] = s0.w;
    c.s[4] = s1.x; c.s[5] = s1.y; c.s[6] = s1.z; c.s[7] = s1.w;
    c.t[0] = h0.x; c.t[1] = h0.y; c.t[2] = h0.z; c.t[3] = h0.w;
    c.t[4] = h1.x; c.t[5] = h1.y; c.t[6] = h1.z; c.t[7] = h1.w;
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) { c.s[k] = 0.f; c.t[k] = 0.f; }
  }
}

// relu(v*scale + shift) on the 8 bf16 of a chunk (same fp32 expression and rounding as the
// BatchNorm apply kernel, so fused and unfused paths agree bit for bit).
__device__ __forceinline__ uint4 affine_relu8(uint4 v, const Coef8& c) {
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float lo = fmaxf(fmaf(__uint_as_float(w[k] << 16), c.s[2 * k], c.t[2 * k]), 0.f);
    const float hi = fmaxf(fmaf(__uint_as_float(w[k] & 0xffff0000u), c.s[2 * k + 1], c.t[2 * k + 1]), 0.f);
    w[k] = (uint32_t)bf16_rne(lo) | ((uint32_t)bf16_rne(hi) << 16);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

template <int R, int BK, bool KC, bool PRO>
__device__ __forceinline__ void store_tile(uint16_t* __restrict__ S,
                                           const uint4 (&r)[Tile<R, BK, KC>::PER_T],
                                           uint32_t okmask, const Coef8& co) {
  using T = Tile<R, BK, KC>;
  static_assert(GT % T::CPR == 0, "chunk column must be constant per thread");
#pragma unroll
  for (int h = 0; h < T::PER_T; ++h) {
    int rr, cc;
    chunk_pos<R, BK, KC>(threadIdx.x + h * GT, rr, cc);
    uint4 v = r[h];
    if (PRO && ((okmask >> h) & 1u)) v = affine_relu8(v, co);
    *reinterpret_cast<uint4*>(S + rr * T::LD + cc * 8) = v;
  }
}

// MFMA operand fragment (8 bf16 along k, k-group g = lane>>4, sub-step s of 32 k) for tile
// row/col i_base + (lane&15).
template <int R, int BK, bool KC>
__device__ __forceinline__ bf16x8 load_frag(const uint16_t* S, int i_base, int s) {
  using T = Tile<R, BK, KC>;
  const int l = threadIdx.x & 63;
  if (KC) {
    const uint16_t* p = S + (i_base + (l & 15)) * T::LD + 32 * s + 8 * (l >> 4);
    return *reinterpret_cast<const bf16x8*>(p);
  } else {
    const int g = l >> 4, t = l & 15, q = t >> 2, p4 = t & 3;
    typedef __attribute__((address_space(3))) i16x4 lds_v4;
    const uint16_t* p0 = S + (32 * s + 8 * g + q) * T::LD + i_base + 4 * p4;
    const uint16_t* p1 = p0 + 4 * T::LD;
    const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(p0));
    const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(p1));
    typedef short i16x8 __attribute__((ext_vector_type(8)));
    const i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

__device__ __forceinline__ void store_out8(void* C, int64_t off, const float v[8], bool bf) {
  if (bf) {
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

struct GemmK {
  const uint16_t* A;
  const uint16_t* B;
  void* C;
  float* partial;
  float* stats;
  const float* bias;
  const float* pro_scale;
  const float* pro_shift;
  const uint16_t* addend;      // optional bf16 [M][ldc] added to a bf16 output (after rounding)
  const uint8_t* add_bits;     // optional ReLU bitmap of the addend (1 bit/element, ldc == N):
                               // the addend enters as addend·[bit] (a BN+ReLU backward's dres)
  int64_t lda, ldb, ldc;
  int M, N, K, k_per_split, relu, out_bf16, accumulate;   // accumulate: fp32 C += result
};

// Workgroup id → (m-tile, n-tile): consecutive ids are dealt round-robin to the 8 XCDs, so remap
// each XCD's share onto one contiguous range of the row-major tile order.
__device__ __forceinline__ int xcd_remap(int pid, int total) {
  const int q = total >> 3, rem = total & 7;
  const int x = pid & 7, idx = pid >> 3;
  return x * q + (x < rem ? x : rem) + idx;
}

template <int BM, int BN, int BK, bool AKC, bool BKC, int EPI, int PRO>
__global__ __launch_bounds__(GT) void k_gemm(const GemmK p) {
  using TA = Tile<BM, BK, AKC>;
  using TB = Tile<BN, BK, BKC>;
  constexpr int WTM = BM / 2, WTN = BN / 2, FM = WTM / 16, FN = WTN / 16;
  constexpr int STAGE = TA::ELEMS + TB::ELEMS;
  constexpr int LDC = BN + 4;                  // fp32 staging row (≡ 4 dwords mod 64 banks)
  constexpr int LDH = BN + 16;                 // bf16 staging row (≡ 8 dwords mod 64 banks)
  constexpr int CS_BYTES = WTM * LDC * 4;
  constexpr int CH_BYTES = BM * LDH * 2 + 2 * 2 * BN * 4;
  constexpr int ST_BYTES = 2 * STAGE * 2;
  constexpr int LDS_BYTES = ST_BYTES > CS_BYTES ? (ST_BYTES > CH_BYTES ? ST_BYTES : CH_BYTES)
                                                : (CS_BYTES > CH_BYTES ? CS_BYTES : CH_BYTES);
  static_assert(PRO != PRO_A || AKC, "PRO_A needs a K-contiguous A");
  static_assert(PRO != PRO_B || !BKC, "PRO_B needs an N-contiguous B");
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
  uint16_t* st = reinterpret_cast<uint16_t*>(lds);

  const int tiles_n = (p.N + BN - 1) / BN, tiles_m = (p.M + BM - 1) / BM;
  const int pid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tm = pid / tiles_n, tn = pid - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = blockIdx.y * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int wr = w >> 1, wc = w & 1;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[TA::PER_T], rb[TB::PER_T];
  int ca[TA::PER_T], cb[TB::PER_T];
  uint32_t oka = 0, okb = 0;
  int cur = 0;
  Coef8 coA, coB;
  if (PRO == PRO_B)        // channel n of this thread's B chunks: fixed for the whole kernel
    load_coef8(coB, p.pro_scale, p.pro_shift, n0 + (threadIdx.x % TB::CPR) * 8, p.N);
  const int a_koff = (threadIdx.x % TA::CPR) * 8;      // PRO_A: k offset within a K-step
  if (kbeg < kend) {
    load_tile<BM, BK, AKC>(p.A, p.lda, m0, p.M, kbeg, kend, ra, ca, oka);
    load_tile<BN, BK, BKC>(p.B, p.ldb, n0, p.N, kbeg, kend, rb, cb, okb);
    if (PRO == PRO_A) load_coef8(coA, p.pro_scale, p.pro_shift, kbeg + a_koff, kend);
    store_tile<BM, BK, AKC, PRO == PRO_A>(st, ra, oka, coA);
    store_tile<BN, BK, BKC, PRO == PRO_B>(st + TA::ELEMS, rb, okb, coB);
  }
  __syncthreads();
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    const bool more = k0 + BK < kend;
    if (more) {
      load_tile<BM, BK, AKC>(p.A, p.lda, m0, p.M, k0 + BK, kend, ra, ca, oka);
      load_tile<BN, BK, BKC>(p.B, p.ldb, n0, p.N, k0 + BK, kend, rb, cb, okb);
      // next stage's prologue coefficients travel with its tile loads (latency hidden by the
      // MFMAs below; coA is free: the current stage was normalised when it was staged)
      if (PRO == PRO_A) load_coef8(coA, p.pro_scale, p.pro_shift, k0 + BK + a_koff, kend);
    }
    const uint16_t* As = st + cur * STAGE;
    const uint16_t* Bs = As + TA::ELEMS;
#pragma unroll
    for (int s = 0; s < BK / 32; ++s) {
      bf16x8 fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = load_frag<BM, BK, AKC>(As, wr * WTM + i * 16, s);
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = load_frag<BN, BK, BKC>(Bs, wc * WTN + j * 16, s);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    if (more) {
      uint16_t* nx = st + (cur ^ 1) * STAGE;
      store_tile<BM, BK, AKC, PRO == PRO_A>(nx, ra, oka, coA);
      store_tile<BN, BK, BKC, PRO == PRO_B>(nx + TA::ELEMS, rb, okb, coB);
    }
    __syncthreads();
    cur ^= 1;
  }

  // ---- epilogue. B is the MFMA's first operand, so each accumulator holds Cᵀ: lane l has
  // C[m = .. + (l&15)][n = .. + 4*(l>>4) + r], r = 0..3 (four consecutive columns of one row).
  const int lm = l & 15, ln = 4 * (l >> 4);
  const bool bf_out = EPI != EPI_PARTIAL && p.out_bf16;
  uint16_t* Ch = reinterpret_cast<uint16_t*>(lds);                  // bf16 tile [BM][LDH]
  float* red = reinterpret_cast<float*>(lds + BM * LDH * 2);        // stats [2 wave rows][2][BN]
  if (EPI != EPI_PARTIAL) {
    // bias / ReLU / rounding in registers; column statistics; bf16 staging of the whole tile
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int nl = wc * WTN + j * 16 + ln;
      const int n = n0 + nl;
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if (p.bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = n + r < p.N ? p.bias[n + r] : 0.f;
      }
      float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int ml = wr * WTM + i * 16 + lm;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float x = acc[i][j][r] + bv[r];
          if (p.relu) x = fmaxf(x, 0.f);
          v[r] = x;
        }
        if (bf_out) {
          uint16_t h[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            h[r] = bf16_rne(v[r]);
            v[r] = __uint_as_float((uint32_t)h[r] << 16);
          }
          *reinterpret_cast<uint2*>(Ch + ml * LDH + nl) =
              make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16));
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] = v[r];
        }
        if (EPI == EPI_STATS && !bf_out && m0 + ml < p.M) {
#pragma unroll
          for (int r = 0; r < 4; ++r) { s1[r] += v[r]; s2[r] += v[r] * v[r]; }
        }
      }
      if (EPI == EPI_STATS && !bf_out) {
        // the 16 rows held by lanes sharing l>>4, fixed butterfly order
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            s1[r] += __shfl_xor(s1[r], o, 64);
            s2[r] += __shfl_xor(s2[r], o, 64);
          }
        }
        if (lm == 0) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            red[(wr * 2 + 0) * BN + nl + r] = s1[r];
            red[(wr * 2 + 1) * BN + nl + r] = s2[r];
          }
        }
      }
    }
  }
  // Column statistics come from the staged bf16 tile during the store pass: a thread's chunks
  // all cover the same 8 columns (GT is a multiple of BN/8), so it sums them in registers and
  // one LDS fold per tile finishes the job (no cross-lane shuffles in the epilogue).
  static_assert(GT % (BN / 8) == 0, "store chunks must keep their column per thread");
  float cs1[8], cs2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { cs1[k] = 0.f; cs2[k] = 0.f; }
  if (bf_out) {
    __syncthreads();
    const bool vec = (p.ldc & 7) == 0;
    for (int c = threadIdx.x; c < BM * (BN / 8); c += GT) {
      const int r = c / (BN / 8), cc = (c % (BN / 8)) * 8;
      const int gm = m0 + r, gn = n0 + cc;
      if (gm >= p.M || gn >= p.N) continue;
      const uint16_t* src = Ch + r * LDH + cc;
      if (EPI == EPI_STATS) {
        const uint4 q = *reinterpret_cast<const uint4*>(src);
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float lo = __uint_as_float(w[k] << 16), hi = __uint_as_float(w[k] & 0xffff0000u);
          const bool in_lo = gn + 2 * k < p.N, in_hi = gn + 2 * k + 1 < p.N;
          cs1[2 * k] += in_lo ? lo : 0.f;
          cs2[2 * k] += in_lo ? lo * lo : 0.f;
          cs1[2 * k + 1] += in_hi ? hi : 0.f;
          cs2[2 * k + 1] += in_hi ? hi * hi : 0.f;
        }
      }
      uint16_t* dst = static_cast<uint16_t*>(p.C) + (int64_t)gm * p.ldc + gn;
      if (vec && gn + 8 <= p.N) {
        uint4 v = *reinterpret_cast<const uint4*>(src);
        if (p.addend) v = add_bf16x8(v, masked_addend8(p.addend, p.add_bits, (int64_t)gm * p.ldc + gn));
        *reinterpret_cast<uint4*>(dst) = v;
      } else {
        for (int k = 0; k < 8 && gn + k < p.N; ++k) {
          uint16_t h = src[k];
          if (p.addend)
            h = bf16_rne(__uint_as_float((uint32_t)h << 16) +
                         masked_addend1(p.addend, p.add_bits, (int64_t)gm * p.ldc + gn + k));
          dst[k] = h;
        }
      }
    }
  } else {
    // fp32 output or split-K slab: two halves through an fp32 staging tile
    float* Cs = reinterpret_cast<float*>(lds);
    float* P = EPI == EPI_PARTIAL ? p.partial + (int64_t)blockIdx.y * p.M * p.N : nullptr;
    float* dstbase = EPI == EPI_PARTIAL ? P : static_cast<float*>(p.C);
    const int64_t ld = EPI == EPI_PARTIAL ? p.N : p.ldc;
    const bool vec = (p.N & 3) == 0 && (ld & 3) == 0;
    float statsave[2] = {0.f, 0.f};
    if (EPI == EPI_STATS) {                      // red[] overlaps Cs: park this thread's column
      __syncthreads();
      for (int c = threadIdx.x; c < BN; c += GT) {
        statsave[0] = red[0 * BN + c] + red[2 * BN + c];
        statsave[1] = red[1 * BN + c] + red[3 * BN + c];
      }
    }
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      __syncthreads();
      if (wr == half) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            *reinterpret_cast<float4*>(Cs + (i * 16 + lm) * LDC + wc * WTN + j * 16 + ln) =
                make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      }
      __syncthreads();
      const int mb = m0 + half * WTM;
      for (int c = threadIdx.x; c < WTM * (BN / 4); c += GT) {
        const int r = c / (BN / 4), cc = (c % (BN / 4)) * 4;
        const int gm = mb + r, gn = n0 + cc;
        if (gm >= p.M || gn >= p.N) continue;
        const float* src = Cs + r * LDC + cc;
        float* dst = dstbase + (int64_t)gm * ld + gn;
        const bool acc_in = EPI != EPI_PARTIAL && p.accumulate;
        if (vec && gn + 4 <= p.N) {
          float4 v = *reinterpret_cast<const float4*>(src);
          if (acc_in) {
            const float4 o = *reinterpret_cast<const float4*>(dst);
            v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
          }
          *reinterpret_cast<float4*>(dst) = v;
        } else {
          for (int k = 0; k < 4 && gn + k < p.N; ++k) dst[k] = acc_in ? dst[k] + src[k] : src[k];
        }
      }
    }
    if (EPI == EPI_STATS) {
      for (int c = threadIdx.x; c < BN; c += GT) {
        const int n = n0 + c;
        if (n >= p.N) continue;
        p.stats[(int64_t)tm * 2 * p.N + n] = statsave[0];
        p.stats[(int64_t)tm * 2 * p.N + p.N + n] = statsave[1];
      }
    }
    return;
  }
  if (EPI == EPI_STATS) {
    // fold the per-thread column sums: GT/(BN/8) threads share each 8-column group
    constexpr int G8 = BN / 8, Q = GT / G8;
    __syncthreads();                              // the staged tile is no longer read
    float* fold = reinterpret_cast<float*>(lds);  // [GT][16]
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
      for (int q = 0; q < Q; ++q) {               // fixed order: deterministic
        a += fold[(q * G8 + g) * 16 + k];
        b += fold[(q * G8 + g) * 16 + 8 + k];
      }
      // [tiles_m][2][N]: one coalesced row per M-tile (bn.hip k_colsum folds the rows)
      p.stats[(int64_t)tm * 2 * p.N + n] = a;
      p.stats[(int64_t)tm * 2 * p.N + p.N + n] = b;
    }
  }
}

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
      uint16_t h = bf16_rne(x);
      if (addend)
        h = bf16_rne(__uint_as_float((uint32_t)h << 16) + masked_addend1(addend, add_bits, m * ldc + n));
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
      const bf16x8 fa0 = __builtin_bit_cast(bf16x8, a_cur[0][s]);
      const bf16x8 fa1 = __builtin_bit_cast(bf16x8, a_cur[1][s]);
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const bf16x8 fb = *reinterpret_cast<const bf16x8*>(
            Bs + (16 * j + (l & 15)) * LDB + 32 * s + 8 * (l >> 4));
        acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb, fa0, acc[0][j], 0, 0, 0);
        acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb, fa1, acc[1][j], 0, 0, 0);
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
        const uint32_t lo = (uint32_t)bf16_rne(acc[i][j][0]) | ((uint32_t)bf16_rne(acc[i][j][1]) << 16);
        const uint32_t hi = (uint32_t)bf16_rne(acc[i][j][2]) | ((uint32_t)bf16_rne(acc[i][j][3]) << 16);
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
          const float lo = __uint_as_float(q[k] << 16), hi = __uint_as_float(q[k] & 0xffff0000u);
          cs1[2 * k] += lo; cs2[2 * k] += lo * lo;
          cs1[2 * k + 1] += hi; cs2[2 * k + 1] += hi * hi;
        }
      }
      uint16_t* dst = static_cast<uint16_t*>(p.C) + (int64_t)gm * p.ldc + gn;
      if (ADD) v = add_bf16x8(v, masked_addend8(p.addend, p.add_bits, (int64_t)gm * p.ldc + gn));
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
static TileShape tile_shape(int t) {
  switch (t) {
    case GEMM_T128x128x64: return {128, 128, 64};
    case GEMM_T256x64x32: return {256, 64, 32};
    case GEMM_T64x256x32: return {64, 256, 32};
    case GEMM_T256x64x64: return {256, 64, 64};
    case GEMM_T64x64x64: return {64, 64, 64};
    default: return {128, 128, 32};
  }
}

int gemm_pick_tile(const GemmArgs& g) {
  if (g.tile > 0) return g.tile;
  if (g.M <= 64 && g.N <= 64) return GEMM_T64x64x64;
  if (g.N <= 64 && g.M >= 512) return GEMM_T256x64x32;
  if (g.M <= 64 && g.N >= 512) return GEMM_T64x256x32;
  return GEMM_T128x128x32;
}

int gemm_tiles_m(const GemmArgs& g) {
  if (g.tile >= GEMM_S64) return gemm_stream_grid_m(g);   // one statistics row per workgroup
  return (g.M + tile_shape(gemm_pick_tile(g)).bm - 1) / tile_shape(gemm_pick_tile(g)).bm;
}

static int k_per_split(int K, int splits, int bk) {
  splits = splits < 1 ? 1 : splits;
  int kps = (K + splits - 1) / splits;
  return (kps + bk - 1) / bk * bk;
}

int gemm_splits_used(const GemmArgs& g) {
  if (g.tile >= GEMM_S64) return 1;
  const int bk = tile_shape(gemm_pick_tile(g)).bk;
  const int kps = k_per_split(g.K, g.splits, bk);
  return (g.K + kps - 1) / kps;
}

template <int BM, int BN, int BK, int EPI, int PRO>
static void launch_layout(const GemmArgs& g, const GemmK& k, dim3 grid, hipStream_t st) {
  const dim3 block(GT);
  if constexpr (PRO == PRO_A) {
    if (g.b_kcontig) hipLaunchKernelGGL((k_gemm<BM, BN, BK, true, true, EPI, PRO>), grid, block, 0, st, k);
    else hipLaunchKernelGGL((k_gemm<BM, BN, BK, true, false, EPI, PRO>), grid, block, 0, st, k);
  } else if constexpr (PRO == PRO_B) {
    if (g.a_kcontig) hipLaunchKernelGGL((k_gemm<BM, BN, BK, true, false, EPI, PRO>), grid, block, 0, st, k);
    else hipLaunchKernelGGL((k_gemm<BM, BN, BK, false, false, EPI, PRO>), grid, block, 0, st, k);
  } else {
    if (g.a_kcontig && g.b_kcontig) hipLaunchKernelGGL((k_gemm<BM, BN, BK, true, true, EPI, PRO>), grid, block, 0, st, k);
    else if (g.a_kcontig) hipLaunchKernelGGL((k_gemm<BM, BN, BK, true, false, EPI, PRO>), grid, block, 0, st, k);
    else if (g.b_kcontig) hipLaunchKernelGGL((k_gemm<BM, BN, BK, false, true, EPI, PRO>), grid, block, 0, st, k);
    else hipLaunchKernelGGL((k_gemm<BM, BN, BK, false, false, EPI, PRO>), grid, block, 0, st, k);
  }
}

template <int BM, int BN, int BK>
static void launch_tile(const GemmArgs& g, const GemmK& k, int epi, dim3 grid, hipStream_t st) {
  const int pro = g.pro_scale ? (g.pro_on_a ? PRO_A : PRO_B) : PRO_NONE;
#define LW_E(E)                                                                                  \
  if (pro == PRO_A) launch_layout<BM, BN, BK, E, PRO_A>(g, k, grid, st);                         \
  else if (pro == PRO_B) launch_layout<BM, BN, BK, E, PRO_B>(g, k, grid, st);                    \
  else launch_layout<BM, BN, BK, E, PRO_NONE>(g, k, grid, st);
  if (epi == EPI_PARTIAL) { LW_E(EPI_PARTIAL) }
  else if (epi == EPI_STATS) { LW_E(EPI_STATS) }
  else { LW_E(EPI_STORE) }
#undef LW_E
}

void gemm_bf16(const GemmArgs& g, hipStream_t st) {
  if (g.tile >= GEMM_S64) {
    gemm_stream(g, st);
    return;
  }
  const int t = gemm_pick_tile(g);
  const TileShape ts = tile_shape(t);
  const int kps = k_per_split(g.K, g.splits, ts.bk);
  const int zs = (g.K + kps - 1) / kps;
  const int tiles = ((g.M + ts.bm - 1) / ts.bm) * ((g.N + ts.bn - 1) / ts.bn);
  const int epi = zs > 1 ? EPI_PARTIAL : (g.stats ? EPI_STATS : EPI_STORE);
  GemmK k{g.A, g.B, g.C, g.partial, g.stats, zs > 1 ? nullptr : g.bias, g.pro_scale, g.pro_shift,
          g.addend, g.add_bits, g.lda, g.ldb, g.ldc, g.M, g.N, g.K, kps, zs > 1 ? 0 : g.relu,
          g.out_bf16 ? 1 : 0, g.accumulate ? 1 : 0};
  const dim3 grid(tiles, zs);
  switch (t) {
    case GEMM_T128x128x64: launch_tile<128, 128, 64>(g, k, epi, grid, st); break;
    case GEMM_T256x64x32: launch_tile<256, 64, 32>(g, k, epi, grid, st); break;
    case GEMM_T64x256x32: launch_tile<64, 256, 32>(g, k, epi, grid, st); break;
    case GEMM_T256x64x64: launch_tile<256, 64, 64>(g, k, epi, grid, st); break;
    case GEMM_T64x64x64: launch_tile<64, 64, 64>(g, k, epi, grid, st); break;
    default: launch_tile<128, 128, 32>(g, k, epi, grid, st); break;
  }
  if (zs > 1) {
    const int64_t total = (int64_t)g.M * g.N;
    int zl = 0;                                  // split lanes: up to 32, no more than splits
    while (zl < 5 && (2 << zl) <= zs) ++zl;
    const int64_t groups = (total + 3) / 4, ot = GT >> zl;
    const dim3 rg((unsigned)((groups + ot - 1) / ot));
    hipLaunchKernelGGL(k_splitk_reduce, rg, dim3(GT), 0, st, g.partial, zs, zl, g.C, g.ldc, g.bias,
                       g.relu, g.M, g.N, g.out_bf16 ? 1 : 0, g.addend, g.add_bits,
                       g.accumulate ? 1 : 0);
  }
}

}  // namespace lw
