// bf16 MFMA GEMM core for gfx950, shared by the plain GEMM (gemm.hip) and the implicit-GEMM
// convolutions (conv.hip): tile staging, MFMA main loop and the fused epilogues.
// See gemm.hip for the design notes.
#pragma once
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
  // loads (or zeros) into locals first, then unconditional member stores: stores in both arms
  // of a branch get sunk into one store through a selected address, which puts the whole
  // struct in scratch memory
  const bool in = j + 8 <= limit;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 s0 = in ? *reinterpret_cast<const float4*>(sc + j) : z;
  const float4 s1 = in ? *reinterpret_cast<const float4*>(sc + j + 4) : z;
  const float4 h0 = in ? *reinterpret_cast<const float4*>(sh + j) : z;
  const float4 h1 = in ? *reinterpret_cast<const float4*>(sh + j + 4) : z;
  c.s[0] = s0.x; c.s[1] = s0.y; c.s[2] = s0.z; c.s[3] = s0.w;
  c.s[4] = s1.x; c.s[5] = s1.y; c.s[6] = s1.z; c.s[7] = s1.w;
  c.t[0] = h0.x; c.t[1] = h0.y; c.t[2] = h0.z; c.t[3] = h0.w;
  c.t[4] = h1.x; c.t[5] = h1.y; c.t[6] = h1.z; c.t[7] = h1.w;
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

// ---- implicit-GEMM convolution geometry (conv.hip). One operand of the GEMM is an im2col
// gather of an NHWC bf16 tensor X[Nb][Hin][Win][C]; the gathered index is a pixel of a "row grid"
// (Hg x Wg per image) and a tap (jr, js) of the class's TR x TS window:
//     hi = y*sh + oh + dh*jr,  wi = x*sw + ow + dw*js          (zero outside X: the padding)
// A-gather (CV_A*): GEMM rows m = (b, y, x), k = (tap, ci)  — forward and data-gradient convs.
// B-gather (CV_B*): GEMM reduction k = (b, y, x), n = (tap, ci) — weight-gradient convs.
// A data-gradient of a stride-2 conv runs as up to 4 parity classes (blockIdx.z) of stride-1
// sub-problems; each class has its own taps, B slab and output row map.
// (gather modes CV_*: lw_kernels.h)

struct ConvClass {
  int TR, TS;           // taps of this class along h / w
  int oh, ow;           // tap origin offsets
  int Hg, Wg;           // row grid per image
  int py, px;           // output row map: pixel (y*osy + py, x*osx + px) of the Hout x Wout grid
  int M, K;             // GEMM rows (A-gather) and reduction length of this class
  int64_t b_off;        // element offset of this class's B operand
};

struct ConvGeom {
  int Hin, Win, C;      // gathered tensor (C = channel count and pixel stride, 4 or a multiple of 8)
  int sh, sw, dh, dw;   // gather stride and tap direction (+1, or -1 for data gradients)
  int Hout, Wout, osy, osx;  // output grid and class strides (row remap when osy*osx > 1)
  int nclass;
  ConvClass cls[4];
};

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
  ConvGeom cv;                 // CV_* kernels only
};

// q = a / d, r = a % d for 0 <= a < 2^24 via the fp32 reciprocal (one correction step each way:
// the estimate is off by at most one) — the per-chunk pixel decode of the gathers.
__device__ __forceinline__ int fdivmod(int a, int d, float inv, int& r) {
  int q = (int)((float)a * inv);
  r = a - q * d;
  if (r < 0) { --q; r += d; }
  else if (r >= d) { ++q; r -= d; }
  return q;
}

// ---- A-gather (im2col rows): per-thread row state, fixed for the whole K loop
template <int R, int BK>
struct RowGather {
  static constexpr int PT = Tile<R, BK, true>::PER_T;
  int base[PT];   // b*Hin*Win, or -1 for rows past the class's M
  int hb[PT], wb[PT];
};

template <int R, int BK>
__device__ __forceinline__ void row_gather_init(RowGather<R, BK>& g, const ConvGeom& cv,
                                                const ConvClass& cc, int m0) {
  using T = Tile<R, BK, true>;
  const int hw = cc.Hg * cc.Wg;
#pragma unroll
  for (int h = 0; h < T::PER_T; ++h) {
    int rr, c8;
    chunk_pos<R, BK, true>(threadIdx.x + h * GT, rr, c8);
    const int m = m0 + rr;
    const bool in = m < cc.M;
    const int mm = in ? m : 0;                   // (branch-free: see load_coef8)
    const int b = mm / hw, rem = mm - b * hw;
    const int y = rem / cc.Wg, x = rem - y * cc.Wg;
    g.base[h] = in ? b * cv.Hin * cv.Win : -1;
    g.hb[h] = y * cv.sh + cc.oh;
    g.wb[h] = x * cv.sw + cc.ow;
  }
}

// K-contiguous A tile of an im2col matrix: chunk = 8 consecutive channels of one pixel and tap
// (C % 8 == 0), or — C4 — two horizontally adjacent taps of a 4-channel pixel (TS even). `ci`
// returns the first channel of each chunk for the BN prologue.
template <int R, int BK, bool C4>
__device__ __forceinline__ void load_tile_gather_a(const uint16_t* __restrict__ X, const ConvGeom& cv,
                                                   const ConvClass& cc, const RowGather<R, BK>& g,
                                                   int k0, int kend,
                                                   uint4 (&r)[Tile<R, BK, true>::PER_T],
                                                   int& ci_out, uint32_t& okmask) {
  using T = Tile<R, BK, true>;
  const int kk = k0 + (threadIdx.x % T::CPR) * 8;   // same for all of this thread's chunks
  int t, ci;
  if (C4) { t = kk >> 2; ci = 0; }
  else { t = kk / cv.C; ci = kk - t * cv.C; }
  const int jr = t / cc.TS, js = t - jr * cc.TS;
  const int hoff = cv.dh * jr, woff = cv.dw * js;
  const bool kin = kk < kend;
  ci_out = ci;
  okmask = 0;
#pragma unroll
  for (int h = 0; h < T::PER_T; ++h) {
    const int hi = g.hb[h] + hoff, wi = g.wb[h] + woff;
    const bool row_ok = kin && g.base[h] >= 0 && (unsigned)hi < (unsigned)cv.Hin;
    if (C4) {
      // pixels wi and wi + dw, 4 channels (8 bytes) each
      const int wi2 = wi + cv.dw;
      const bool ok0 = row_ok && (unsigned)wi < (unsigned)cv.Win;
      const bool ok1 = row_ok && (unsigned)wi2 < (unsigned)cv.Win;
      const int64_t rowpix = (int64_t)g.base[h] + (int64_t)hi * cv.Win;
      const uint2 a = ok0 ? *reinterpret_cast<const uint2*>(X + (rowpix + wi) * 4) : make_uint2(0, 0);
      const uint2 b = ok1 ? *reinterpret_cast<const uint2*>(X + (rowpix + wi2) * 4) : make_uint2(0, 0);
      r[h] = make_uint4(a.x, a.y, b.x, b.y);
      okmask |= (ok0 || ok1 ? 1u : 0u) << h;
    } else {
      const bool ok = row_ok && (unsigned)wi < (unsigned)cv.Win;
      const int64_t off = ((int64_t)g.base[h] + (int64_t)hi * cv.Win + wi) * cv.C + ci;
      r[h] = ok ? *reinterpret_cast<const uint4*>(X + off) : make_uint4(0, 0, 0, 0);
      okmask |= (ok ? 1u : 0u) << h;
    }
  }
}

// ---- B-gather (weight gradient): N-contiguous B tile whose rows are pixels of the output grid
// and whose chunks are (tap, 8 channels) — or C4: (tap pair, 4 channels) — of the input.
struct ColGather {
  int hoff, woff, ci;   // tap offsets (origin included) and first channel of this thread's chunk
  bool ok;
};

template <int R, int BK, bool C4>
__device__ __forceinline__ void col_gather_init(ColGather& g, const ConvGeom& cv, const ConvClass& cc,
                                                int n0, int N) {
  using T = Tile<R, BK, false>;
  const int nn = n0 + (threadIdx.x % T::CPR) * 8;
  int t, ci;
  if (C4) { t = nn >> 2; ci = 0; }
  else { t = nn / cv.C; ci = nn - t * cv.C; }
  const int jr = t / cc.TS, js = t - jr * cc.TS;
  g.hoff = cc.oh + cv.dh * jr;
  g.woff = cc.ow + cv.dw * js;
  g.ci = ci;
  g.ok = nn < N;
}

template <int R, int BK, bool C4>
__device__ __forceinline__ void load_tile_gather_b(const uint16_t* __restrict__ X, const ConvGeom& cv,
                                                   const ConvClass& cc, const ColGather& g,
                                                   int hw, float inv_hw, float inv_w, int k0,
                                                   int kend, uint4 (&r)[Tile<R, BK, false>::PER_T],
                                                   uint32_t& okmask) {
  using T = Tile<R, BK, false>;
  okmask = 0;
#pragma unroll
  for (int h = 0; h < T::PER_T; ++h) {
    int rr, c8;
    chunk_pos<R, BK, false>(threadIdx.x + h * GT, rr, c8);
    const int pix = k0 + rr;
    int rem, x;
    const int b = fdivmod(pix, hw, inv_hw, rem);
    const int y = fdivmod(rem, cc.Wg, inv_w, x);
    const int hi = y * cv.sh + g.hoff, wi = x * cv.sw + g.woff;
    const bool row_ok = g.ok && pix < kend && (unsigned)hi < (unsigned)cv.Hin;
    const int64_t rowpix = (int64_t)b * cv.Hin * cv.Win + (int64_t)hi * cv.Win;
    if (C4) {
      const int wi2 = wi + cv.dw;
      const bool ok0 = row_ok && (unsigned)wi < (unsigned)cv.Win;
      const bool ok1 = row_ok && (unsigned)wi2 < (unsigned)cv.Win;
      const uint2 a = ok0 ? *reinterpret_cast<const uint2*>(X + (rowpix + wi) * 4) : make_uint2(0, 0);
      const uint2 c = ok1 ? *reinterpret_cast<const uint2*>(X + (rowpix + wi2) * 4) : make_uint2(0, 0);
      r[h] = make_uint4(a.x, a.y, c.x, c.y);
      okmask |= (ok0 || ok1 ? 1u : 0u) << h;
    } else {
      const bool ok = row_ok && (unsigned)wi < (unsigned)cv.Win;
      r[h] = ok ? *reinterpret_cast<const uint4*>(X + (rowpix + wi) * cv.C + g.ci)
                : make_uint4(0, 0, 0, 0);
      okmask |= (ok ? 1u : 0u) << h;
    }
  }
}

// Workgroup id → (m-tile, n-tile): consecutive ids are dealt round-robin to the 8 XCDs, so remap
// each XCD's share onto one contiguous range of the row-major tile order.
__device__ __forceinline__ int xcd_remap(int pid, int total) {
  const int q = total >> 3, rem = total & 7;
  const int x = pid & 7, idx = pid >> 3;
  return x * q + (x < rem ? x : rem) + idx;
}

template <int BM, int BN, int BK, bool AKC, bool BKC, int EPI, int PRO, int CV = CV_NONE>
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
  constexpr bool GA = CV == CV_A || CV == CV_A4, GB = CV == CV_B || CV == CV_B4;
  constexpr bool G4 = CV == CV_A4 || CV == CV_B4;
  static_assert(PRO != PRO_A || AKC, "PRO_A needs a K-contiguous A");
  static_assert(PRO != PRO_B || !BKC, "PRO_B needs an N-contiguous B");
  static_assert(!GA || AKC, "the im2col A gather stages a K-contiguous tile");
  static_assert(!GB || !BKC, "the im2col B gather stages an N-contiguous tile");
  static_assert(!G4 || PRO == PRO_NONE, "4-channel gathers have no BN prologue");
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
  uint16_t* st = reinterpret_cast<uint16_t*>(lds);

  const int tiles_n = (p.N + BN - 1) / BN, tiles_m = (p.M + BM - 1) / BM;
  const int pid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tm = pid / tiles_n, tn = pid - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  // the class record by constant index (a runtime index into the by-value kernel argument
  // would copy the whole array to scratch)
  const int zc = GA ? (int)blockIdx.z : 0;
  const ConvClass ccl = zc == 0 ? p.cv.cls[0] : zc == 1 ? p.cv.cls[1]
                      : zc == 2 ? p.cv.cls[2] : p.cv.cls[3];
  if (GA && m0 >= ccl.M) return;                // parity class with fewer rows than the grid
  const int Kc = GA ? ccl.K : p.K;
  const int kbeg = blockIdx.y * p.k_per_split;
  const int kend = min(Kc, kbeg + p.k_per_split);
  const uint16_t* Bp = GA ? p.B + ccl.b_off : p.B;
  const int Mrow = GA ? ccl.M : p.M;             // valid GEMM rows of this workgroup
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
  RowGather<BM, BK> rg;
  ColGather colg;
  int g_hw = 1;
  float g_inv_hw = 1.f, g_inv_w = 1.f;
  if constexpr (GA) row_gather_init<BM, BK>(rg, p.cv, ccl, m0);
  if constexpr (GB) {
    col_gather_init<BN, BK, G4>(colg, p.cv, ccl, n0, p.N);
    g_hw = ccl.Hg * ccl.Wg;
    g_inv_hw = 1.f / (float)g_hw;
    g_inv_w = 1.f / (float)ccl.Wg;
  }
  if (PRO == PRO_B)        // channel n of this thread's B chunks: fixed for the whole kernel
    load_coef8(coB, p.pro_scale, p.pro_shift,
               GB ? colg.ci : n0 + (threadIdx.x % TB::CPR) * 8, GB ? p.cv.C : p.N);
  const int a_koff = (threadIdx.x % TA::CPR) * 8;      // PRO_A: k offset within a K-step
  // global -> registers for the K-step at k (and, PRO_A, its prologue coefficients)
  auto fetch = [&](int k) {
    int a_ch = k + a_koff;
    if constexpr (GA) load_tile_gather_a<BM, BK, G4>(p.A, p.cv, ccl, rg, k, kend, ra, a_ch, oka);
    else load_tile<BM, BK, AKC>(p.A, p.lda, m0, p.M, k, kend, ra, ca, oka);
    if constexpr (GB)
      load_tile_gather_b<BN, BK, G4>(Bp, p.cv, ccl, colg, g_hw, g_inv_hw, g_inv_w, k, kend, rb, okb);
    else load_tile<BN, BK, BKC>(Bp, p.ldb, n0, p.N, k, kend, rb, cb, okb);
    if (PRO == PRO_A) load_coef8(coA, p.pro_scale, p.pro_shift, a_ch, GA ? p.cv.C : kend);
  };
  if (kbeg < kend) {
    fetch(kbeg);
    store_tile<BM, BK, AKC, PRO == PRO_A>(st, ra, oka, coA);
    store_tile<BN, BK, BKC, PRO == PRO_B>(st + TA::ELEMS, rb, okb, coB);
  }
  __syncthreads();
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    const bool more = k0 + BK < kend;
    // next stage's tiles (and prologue coefficients) travel during the MFMAs below; coA is
    // free: the current stage was normalised when it was staged
    if (more) fetch(k0 + BK);
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
        if (EPI == EPI_STATS && !bf_out && m0 + ml < Mrow) {
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
      if (gm >= Mrow || gn >= p.N) continue;
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
      int64_t orow = gm;
      if (GA && (p.cv.osy > 1 || p.cv.osx > 1)) {   // parity class -> its pixels of the output
        const int hw = ccl.Hg * ccl.Wg, b = gm / hw, rem = gm - b * hw;
        const int y = rem / ccl.Wg, x = rem - y * ccl.Wg;
        orow = ((int64_t)b * p.cv.Hout + y * p.cv.osy + ccl.py) * p.cv.Wout + x * p.cv.osx + ccl.px;
      }
      uint16_t* dst = static_cast<uint16_t*>(p.C) + orow * p.ldc + gn;
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
    float* P = EPI == EPI_PARTIAL ? p.partial + (int64_t)blockIdx.y * Mrow * p.N : nullptr;
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
        if (gm >= Mrow || gn >= p.N) continue;
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

}  // namespace lw
