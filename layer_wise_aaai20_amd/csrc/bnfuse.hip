// BatchNorm-backward apply fused with BOTH GEMMs that consume its output, for the BN3 of the
// ResNet-50 bottlenecks of stages 1 and 2 (c3: CO = 256 / 512 channels, a2: CI = 64 / 128), gfx950.
//
// The per-layer path (ops/block.py) runs, after BN3's reduce + finalize:
//   dc3 = A·(dr·bit) + B·c3 + C          k_bn_bwd_apply  reads dr, c3, bits; writes dc3 (CO ch)
//   dW3 += dc3ᵀ · a2                     GEMM            reads dc3 again (+ a2)
//   da2  = dc3 · W3                      GEMM            reads dc3 a third time, writes da2
// i.e. five CO-channel activation streams (411 / 205 MB each at batch 256). Here one persistent
// kernel reads dr, c3 and the bitmap ONCE per BM-pixel tile, forms the bf16 dc3 tile in LDS (the
// apply's exact expression and rounding) and feeds both products from that LDS image:
//   da2 tile [BM px][64]   = dc3 tile · W3[:, part]  (that W3ᵀ part resident in LDS, K = CO)
//   dW3 [CO][64 of part]  += dc3 tileᵀ · a2 tile    (accumulated in registers across the tiles of
//                                                    the workgroup, K = pixels; one fp32 slab per
//                                                    tile group, summed in fixed order by the
//                                                    split-K reduce, gemm.hip)
// A workgroup owns one 64-column part of CI (stage 2: two parts); the parts of a tile group are
// dealt to blocks b, b + 8, ... so they share an XCD and the second reads dr / c3 from its L2.
// Stage 1: 608.7 -> 410.4 us a block (profiles/r6/fused_bn3/).
//
// LDS images (bf16, 16-byte chunks XOR-swizzled by row so that every fragment read is
// bank-conflict-free):
//   W3ᵀ part [64 ci][CO] and dc3 [BM px][CO]: rows of 2·CO bytes, chunk c at c ^ s512(row), read
//     by rows with ds_read_b128 (16 rows x chunks 2k, 2k+1 per 16-lane group: distinct bank
//     quads) and, for dc3, by columns with ds_read_b64_tr_b16 (the A operand dc3ᵀ of dW3: rows
//     8g+q of chunks 2k, 2k+1 per 32-lane half, s512(row) >> 1 distinct);
//   a2 part [BM px][64 ci]: 128-B rows, chunk c at c ^ s128(row), read by columns (B of dW3);
//   da2 staging [BM px][64 ci] for 16-byte global stores.
// Waves (4, 256 threads, one workgroup per CU): da2 ci rows 16w..16w+15 x BM px; dW3 co rows
// CO/4·w .. +CO/4 x the part's 64 ci.
#include "gemm_core.h"

namespace lw {

namespace {
constexpr int BF_CIP = 64;                // a2 / da2 / W3ᵀ columns per workgroup (one part)

__device__ __forceinline__ int s512(int r) { return ((r & 3) << 1) | (r & 8); }
__device__ __forceinline__ int s128(int r) { return (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2); }

typedef __attribute__((address_space(3))) i16x4 lds_v4;
__device__ __forceinline__ i16x4 tr_read(const uint8_t* a) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)a);
}
__device__ __forceinline__ h16x8 cat8(i16x4 lo, i16x4 hi) {
  typedef short i16x8 __attribute__((ext_vector_type(8)));
  const i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(h16x8, v);
}

// 8 bf16 values with those whose bit of `b` is clear zeroed (the ReLU-masked addend)
__device__ __forceinline__ uint4 mask_h16x8(uint4 a, uint32_t b) {
  const uint32_t m0 = ((b & 1u) ? 0xffffu : 0u) | ((b & 2u) ? 0xffff0000u : 0u);
  const uint32_t m1 = ((b & 4u) ? 0xffffu : 0u) | ((b & 8u) ? 0xffff0000u : 0u);
  const uint32_t m2 = ((b & 16u) ? 0xffffu : 0u) | ((b & 32u) ? 0xffff0000u : 0u);
  const uint32_t m3 = ((b & 64u) ? 0xffffu : 0u) | ((b & 128u) ? 0xffff0000u : 0u);
  return make_uint4(a.x & m0, a.y & m1, a.z & m2, a.w & m3);
}

template <int CO> struct BfGeom {
  static constexpr int BM = CO == 256 ? 64 : 32;        // pixels per tile
  static constexpr int CPR = CO / 8;                    // 16-byte chunks per dc3 row
  static constexpr int RSTEP = 256 / CPR;               // rows between one thread's chunks
  static constexpr int NROW = BM / RSTEP;               // chunks per thread per tile (8)
  static constexpr int NA = BM * 8 / 256;               // a2 chunks per thread per tile
  static constexpr int NCB = CO / 64;                   // dW3 16-row blocks per wave
  static constexpr int W_BYTES = BF_CIP * CO * 2, D_BYTES = BM * CO * 2, A_BYTES = BM * 128;
  static constexpr int LDS = W_BYTES + D_BYTES + 2 * A_BYTES;
};
}  // namespace

// One tile's loads (registers): dy, c3 (and the shortcut's x2) rows, the bitmap bytes, a2 rows
template <int CO> struct BfRaw {
  uint4 d[BfGeom<CO>::NROW], x[BfGeom<CO>::NROW], x2[BfGeom<CO>::NROW], a[BfGeom<CO>::NA];
  uint32_t b[BfGeom<CO>::NROW];
  uint2 c2[BfGeom<CO>::BM / 16];          // S2: c2 at this lane's 4 da2 channels, per pixel block
};

// DUAL: the downsample block, whose shortcut BN (input x2 = cd) received the same dy and ReLU
// bitmap: dx2 = A2·(dy·bit) + B2·x2 + C2 is formed in the same pass and written out (it feeds the
// shortcut's weight and data gradients; with two parts, by the part-0 workgroup). One tile of
// loads is in flight while a tile computes (a second register set, two tiles in flight, measured
// 435.8 vs 420.4 us at stage 1: profiles/r6/fused_bn3/).
// acc_out: a single tile group adds its dW3 straight into `slab` (= the destination).
// S2: BN2's backward reduction rides on the da2 tile: with c2 (BN2's input), its forward affine
// ss2 (scale | shift: the ReLU mask) and mean2, each workgroup adds (Σd, Σd·(c2 − mean2)) of
// d = da2·[c2·s + h > 0] over its pixels — k_bn_reduce RELU 2's expression on the same bf16 da2
// values — and writes them as row `grp` of st2 [groups][2][CI] (its part's 64 columns), which
// the BN2 finalize folds in place: the separate reduce pass over da2 and c2 is gone.
// A2C: `a2` is c2 itself and the kernel forms a2 = relu(c2·s + h) (bf16, k_bn_apply's expression)
// as it stages the tile — the forward then never materialises a2 (its GEMM applies BN2 in the
// prologue), and the tile's c2 bytes are the ones S2 reads.
template <int CO, bool DUAL, bool S2, bool A2C>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1)))
void k_bn3_bwd_dgemm(const uint16_t* __restrict__ dr, const uint16_t* __restrict__ c3,
                     const uint8_t* __restrict__ bits, const float* __restrict__ A,
                     const float* __restrict__ B, const float* __restrict__ Cc,
                     const uint16_t* __restrict__ w3t, const uint16_t* __restrict__ a2,
                     uint16_t* __restrict__ da2, float* __restrict__ slab,
                     const uint16_t* __restrict__ x2, const float* __restrict__ A2,
                     const float* __restrict__ B2, const float* __restrict__ C2,
                     uint16_t* __restrict__ dx2, const uint16_t* __restrict__ c2,
                     const float* __restrict__ ss2, const float* __restrict__ mean2,
                     float* __restrict__ st2, int64_t M, int CI, int tiles, int tpw,
                     int acc_out, int xcd_pairs) {
  using G = BfGeom<CO>;
  constexpr int BM = G::BM, RB = CO * 2;              // dc3 / W3ᵀ row bytes
  __shared__ __attribute__((aligned(16))) uint8_t lds[G::LDS];
  uint8_t* const sW = lds;                            // W3ᵀ part [64][RB]
  uint8_t* const sD = lds + G::W_BYTES;               // dc3      [BM][RB]
  uint8_t* const sA = sD + G::D_BYTES;                // a2 part  [BM][128 B]
  uint8_t* const sO = sA + G::A_BYTES;                // da2      [BM][128 B]
  const int t = threadIdx.x, l = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int g = l >> 4, q = (l & 15) >> 2, p = l & 3;
  // block -> (tile group, part): with a multiple of 8 groups the parts of one group are blocks 8
  // apart (one XCD under round-robin placement: speed only), else consecutive
  const int nparts = CI / BF_CIP;
  const int bx = (int)blockIdx.x & 7, by = (int)blockIdx.x >> 3;
  const int part = xcd_pairs ? by % nparts : (int)blockIdx.x % nparts;
  const int grp = xcd_pairs ? (by / nparts) * 8 + bx : (int)blockIdx.x / nparts;
  const int c0 = part * BF_CIP;
  const int u0 = grp * tpw, u1 = min(u0 + tpw, tiles);
  const bool write_dx2 = DUAL && part == 0;
  const uint32_t act_bytes = (uint32_t)(M * CO * 2), a2_bytes = (uint32_t)(M * CI * 2);
  const __amdgpu_buffer_rsrc_t rdr = make_rsrc(dr, act_bytes), rc3 = make_rsrc(c3, act_bytes);
  const __amdgpu_buffer_rsrc_t rx2 = make_rsrc(DUAL ? x2 : c3, act_bytes);
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(a2, a2_bytes);
  const __amdgpu_buffer_rsrc_t rc2 = make_rsrc(S2 ? c2 : a2, a2_bytes);
  Coef8 co2;                                           // A2C: BN2 of this thread's a2 chunk column
  if (A2C) load_coef8(co2, ss2, ss2 + CI, c0 + (t & 7) * 8, CI);
  // S2: this lane's da2 channels ci2 .. ci2 + 3 (the staging layout below) and their BN2 terms
  const int ci2 = c0 + 16 * w + 4 * g;
  float fs2[4], fh2[4], mu2[4], st_a[4], st_b[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    fs2[r] = S2 ? ss2[ci2 + r] : 0.f;
    fh2[r] = S2 ? ss2[CI + ci2 + r] : 0.f;
    mu2[r] = S2 ? mean2[ci2 + r] : 0.f;
    st_a[r] = 0.f;
    st_b[r] = 0.f;
  }

  // ---- this part's W3ᵀ rows into LDS (once)
#pragma unroll
  for (int i = 0; i < BF_CIP * G::CPR / 256; ++i) {
    const int e = t + 256 * i, row = e / G::CPR, ch = e % G::CPR;
    const uint4 v = *reinterpret_cast<const uint4*>(w3t + (int64_t)(c0 + row) * CO + ch * 8);
    *reinterpret_cast<uint4*>(sW + row * RB + ((ch ^ s512(row & 15)) << 4)) = v;
  }
  // ---- this thread's 8 channels of the apply: chunk column cc, rows prow + RSTEP·i
  const int cc = t % G::CPR, prow = t / G::CPR;
  float ca[8], cb[8], ck[8], ca2[8], cb2[8], ck2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    ca[k] = A[cc * 8 + k]; cb[k] = B[cc * 8 + k]; ck[k] = Cc[cc * 8 + k];
    ca2[k] = DUAL ? A2[cc * 8 + k] : 0.f;
    cb2[k] = DUAL ? B2[cc * 8 + k] : 0.f;
    ck2[k] = DUAL ? C2[cc * 8 + k] : 0.f;
  }

  auto load_tile = [&](int u, BfRaw<CO>& R) {
    const int64_t m0 = (int64_t)u * BM;
#pragma unroll
    for (int i = 0; i < G::NROW; ++i) {
      const int64_t m = m0 + prow + G::RSTEP * i;
      const uint32_t off = m < M ? (uint32_t)((m * CO + cc * 8) * 2) : OOB;
      R.d[i] = bload16(rdr, off);
      R.x[i] = bload16(rc3, off);
      if (DUAL) R.x2[i] = bload16(rx2, off);
      R.b[i] = m < M ? (uint32_t)bits[m * (CO / 8) + cc] : 0u;
    }
#pragma unroll
    for (int i = 0; i < G::NA; ++i) {
      const int e = t + 256 * i;
      const int64_t m = m0 + (e >> 3);
      R.a[i] = bload16(ra, m < M ? (uint32_t)((m * CI + c0 + (e & 7) * 8) * 2) : OOB);
    }
    if (S2) {
#pragma unroll
      for (int j = 0; j < BM / 16; ++j) {
        const int64_t m = m0 + 16 * j + (l & 15);
        R.c2[j] = bload8(rc2, m < M ? (uint32_t)((m * CI + ci2) * 2) : OOB);
      }
    }
  };

  f32x4 acc2[G::NCB][4];
#pragma unroll
  for (int i = 0; i < G::NCB; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- phase A: dc3 = A·(dy·bit) + B·c3 + C (bf16; k_bn_bwd_apply's expression) and a2 into
  // their LDS images (DUAL: dx2 straight to memory)
  auto phase_a = [&](int u, const BfRaw<CO>& R) {
    const int64_t m0 = (int64_t)u * BM;
#pragma unroll
    for (int i = 0; i < G::NROW; ++i) {
      const uint32_t dw[4] = {R.d[i].x, R.d[i].y, R.d[i].z, R.d[i].w};
      const uint32_t xw[4] = {R.x[i].x, R.x[i].y, R.x[i].z, R.x[i].w};
      const uint32_t x2w[4] = {R.x2[i].x, R.x2[i].y, R.x2[i].z, R.x2[i].w};
      uint32_t o[4], o2[4];
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2) {
        float d0 = hlo(dw[k2]), d1 = hhi(dw[k2]);
        d0 = ((R.b[i] >> (2 * k2)) & 1u) ? d0 : 0.f;
        d1 = ((R.b[i] >> (2 * k2 + 1)) & 1u) ? d1 : 0.f;
        const float v0 = ca[2 * k2] * d0 + cb[2 * k2] * hlo(xw[k2]) + ck[2 * k2];
        const float v1 = ca[2 * k2 + 1] * d1 + cb[2 * k2 + 1] * hhi(xw[k2]) + ck[2 * k2 + 1];
        o[k2] = (uint32_t)f2h(v0) | ((uint32_t)f2h(v1) << 16);
        if (DUAL) {
          const float e0 = ca2[2 * k2] * d0 + cb2[2 * k2] * hlo(x2w[k2]) + ck2[2 * k2];
          const float e1 = ca2[2 * k2 + 1] * d1 + cb2[2 * k2 + 1] * hhi(x2w[k2]) + ck2[2 * k2 + 1];
          o2[k2] = (uint32_t)f2h(e0) | ((uint32_t)f2h(e1) << 16);
        }
      }
      const int row = prow + G::RSTEP * i;
      *reinterpret_cast<uint4*>(sD + row * RB + ((cc ^ s512(row & 15)) << 4)) =
          make_uint4(o[0], o[1], o[2], o[3]);
      if (write_dx2 && m0 + row < M)
        *reinterpret_cast<uint4*>(dx2 + (m0 + row) * CO + cc * 8) =
            make_uint4(o2[0], o2[1], o2[2], o2[3]);
    }
#pragma unroll
    for (int i = 0; i < G::NA; ++i) {
      const int e = t + 256 * i, row = e >> 3, ch = e & 7;
      uint4 v = R.a[i];
      // (rows past M stay zero: their dc3 rows are C, not zero)
      if (A2C) v = m0 + row < M ? affine_relu8(v, co2) : make_uint4(0u, 0u, 0u, 0u);
      *reinterpret_cast<uint4*>(sA + row * 128 + ((ch ^ s128(row & 15)) << 4)) = v;
    }
  };

  // ---- phase B: both products from the LDS images, da2 staged and stored
  auto phase_b = [&](int u, const uint2 (&cx)[BM / 16]) {
    // da2 tile: D[ci 16w..][px] = W3ᵀ[ci][co] · dc3[px][co]ᵀ, K = CO channels
    f32x4 acc1[BM / 16];
#pragma unroll
    for (int j = 0; j < BM / 16; ++j) acc1[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int ci_r = 16 * w + (l & 15);
#pragma unroll
    for (int ks = 0; ks < CO / 32; ++ks) {
      const int ch = 4 * ks + g;
      const h16x8 fa = *reinterpret_cast<const h16x8*>(sW + ci_r * RB + ((ch ^ s512(ci_r & 15)) << 4));
#pragma unroll
      for (int j = 0; j < BM / 16; ++j) {
        const int px = 16 * j + (l & 15);
        const h16x8 fb = *reinterpret_cast<const h16x8*>(sD + px * RB + ((ch ^ s512(px & 15)) << 4));
        acc1[j] = mfma16(fa, fb, acc1[j]);
      }
    }
    // dW3[co CO/4·w ..][ci] += dc3ᵀ[co][px] · a2[px][ci], K = BM pixels (transposing reads)
#pragma unroll
    for (int kk = 0; kk < BM / 32; ++kk) {
      i16x4 ta[2][G::NCB], tb[2][4];     // [rows 8g+q / 8g+4+q][block]
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int px = 32 * kk + 8 * g + q + 4 * hh;
        const uint8_t* rowD = sD + px * RB;
        const uint8_t* rowA = sA + px * 128;
#pragma unroll
        for (int i = 0; i < G::NCB; ++i) {
          const int chd = 2 * (G::NCB * w + i) + (p >> 1);
          ta[hh][i] = tr_read(rowD + ((chd ^ s512(px & 15)) << 4) + 8 * (p & 1));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int cha = 2 * j + (p >> 1);
          tb[hh][j] = tr_read(rowA + ((cha ^ s128(px & 15)) << 4) + 8 * (p & 1));
        }
      }
      h16x8 fb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = cat8(tb[0][j], tb[1][j]);
#pragma unroll
      for (int i = 0; i < G::NCB; ++i) {
        const h16x8 fa = cat8(ta[0][i], ta[1][i]);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc2[i][j] = mfma16(fa, fb[j], acc2[i][j]);
      }
    }
    // da2 tile -> staging (lane: ci 16w + 4g .. +3 of pixel 16j + (l & 15))
#pragma unroll
    for (int j = 0; j < BM / 16; ++j) {
      const int px = 16 * j + (l & 15);
      const int ch = 2 * w + (g >> 1);
      uint16_t h[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) h[r] = f2h(acc1[j][r]);
      if (S2 && (int64_t)u * BM + px < M) {
        const uint32_t xw[2] = {cx[j].x, cx[j].y};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float xv = (r & 1) ? hhi(xw[r >> 1]) : hlo(xw[r >> 1]);
          const float d = fmaf(xv, fs2[r], fh2[r]) > 0.f ? h2f(h[r]) : 0.f;
          st_a[r] += d;
          st_b[r] += d * (xv - mu2[r]);
        }
      }
      *reinterpret_cast<uint2*>(sO + px * 128 + ((ch ^ s128(px & 15)) << 4) + 8 * (g & 1)) =
          make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16));
    }
    __syncthreads();
    const int64_t m0 = (int64_t)u * BM;
#pragma unroll
    for (int i = 0; i < G::NA; ++i) {
      const int e = t + 256 * i, row = e >> 3, ch = e & 7;
      if (m0 + row < M)
        *reinterpret_cast<uint4*>(da2 + (m0 + row) * CI + c0 + ch * 8) =
            *reinterpret_cast<const uint4*>(sO + row * 128 + ((ch ^ s128(row & 15)) << 4));
    }
  };

  BfRaw<CO> R0;
  if (u0 < u1) load_tile(u0, R0);
  for (int u = u0; u < u1; ++u) {
    phase_a(u, R0);
    uint2 cx[BM / 16];
#pragma unroll
    for (int j = 0; j < BM / 16; ++j) cx[j] = R0.c2[j];
    __syncthreads();
    if (u + 1 < u1) load_tile(u + 1, R0);      // in flight under this tile's MFMAs
    phase_b(u, cx);
  }
  if (S2) {
    // the 16 lanes of one k group hold the same 4 channels: fixed butterfly, lane 16g writes
#pragma unroll
    for (int o = 1; o < 16; o <<= 1)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        st_a[r] += __shfl_xor(st_a[r], o, 64);
        st_b[r] += __shfl_xor(st_b[r], o, 64);
      }
    if ((l & 15) == 0) {
      float* row = st2 + (int64_t)grp * 2 * CI;
      *reinterpret_cast<float4*>(row + ci2) = make_float4(st_a[0], st_a[1], st_a[2], st_a[3]);
      *reinterpret_cast<float4*>(row + CI + ci2) = make_float4(st_b[0], st_b[1], st_b[2], st_b[3]);
    }
  }
  // ---- this group's dW3 slab (the part's columns): lane holds
  // D[co = (NCB·w + i)·16 + 4g + r][ci = c0 + 16j + (l & 15)]
  float* sl = slab + (int64_t)grp * CO * CI;
#pragma unroll
  for (int i = 0; i < G::NCB; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float* d = sl + (int64_t)((G::NCB * w + i) * 16 + 4 * g + r) * CI + c0 + 16 * j + (l & 15);
        *d = acc_out ? *d + acc2[i][j][r] : acc2[i][j][r];
      }
}

static int bf_tiles(int64_t M, int CO) {
  const int bm = CO == 256 ? BfGeom<256>::BM : BfGeom<512>::BM;
  return (int)((M + bm - 1) / bm);
}

// tile groups (= dW3 slabs): a multiple of 8 (the parts of a group share an XCD), about one
// workgroup per CU over all parts
int bn3_bwd_dgemm_slabs(int64_t M, int C, int Ci) {
  const int tiles = bf_tiles(M, C), nparts = Ci / BF_CIP;
  int want = std::max(8, cu_count() / nparts / 8 * 8);
  const int tpw = (tiles + want - 1) / want;
  const int used = (tiles + tpw - 1) / tpw;
  return used <= 1 ? 1 : (used + 7) / 8 * 8;
}

bool bn3_bwd_dgemm_ok(int64_t M, int C, int Ci) {
  return ((C == 256 && Ci == 64) || (C == 512 && Ci == 128)) && M > 0 &&
         M * C * 2 < (int64_t(1) << 31);
}

void bn3_bwd_dgemm(const uint16_t* dr, const uint16_t* c3, const uint8_t* bits, const float* A,
                   const float* B, const float* Cc, const uint16_t* w3t, const uint16_t* a2,
                   uint16_t* da2, float* slab, int64_t M, int C, int Ci, hipStream_t st,
                   const uint16_t* x2, const float* A2, const float* B2, const float* C2,
                   uint16_t* dx2, bool acc_out, const uint16_t* c2, const float* ss2,
                   const float* mean2, float* st2, bool a2c) {
  const int tiles = bf_tiles(M, C), nparts = Ci / BF_CIP;
  const int groups = bn3_bwd_dgemm_slabs(M, C, Ci);
  const int tpw = (tiles + groups - 1) / groups;
  const int acc = (acc_out && groups == 1) ? 1 : 0;
  const int blocks = groups * nparts, xp = groups % 8 == 0 ? 1 : 0;
#define LW_BF(CO, DU, S, AC)                                                                     \
  hipLaunchKernelGGL((k_bn3_bwd_dgemm<CO, DU, S, AC>), dim3(blocks), dim3(256), 0, st, dr, c3,  \
                     bits, A, B, Cc, w3t, a2, da2, slab, x2, A2, B2, C2, dx2, c2, ss2, mean2,   \
                     st2, M, Ci, tiles, tpw, acc, xp)
#define LW_BF2(CO, DU)                                                                           \
  if (st2) { if (a2c) LW_BF(CO, DU, true, true); else LW_BF(CO, DU, true, false); }               \
  else { if (a2c) LW_BF(CO, DU, false, true); else LW_BF(CO, DU, false, false); }
  if (C == 256) { if (x2) { LW_BF2(256, true); } else { LW_BF2(256, false); } }
  else { if (x2) { LW_BF2(512, true); } else { LW_BF2(512, false); } }
#undef LW_BF2
#undef LW_BF
}

// ---------------------------------------------------------------------------------------------
// The same fusion for BN1 of a bottleneck without a downsample branch (stages 1 and 2): after
// BN1's reduce + finalize, the per-layer path runs
//   dc1 = A·(da1·[c1·s+h > 0]) + B·c1 + C      k_bn_bwd_apply   reads da1, c1; writes dc1 (W ch)
//   dW1 += dc1ᵀ · x                             GEMM             reads dc1, x (Cin ch)
//   dx   = dc1 · W1 + dy·bit3                   GEMM             reads dc1, dy, bitmap; writes dx
// Here dc1 is formed per 64-pixel tile in LDS and feeds both products:
//   dx tile [64 px][Cin part] = dc1 tile · W1[:, part] + dy·bit3   (W1ᵀ part resident in LDS)
//   dW1 [W][Cin part]        += dc1 tileᵀ · x tile                 (registers, slab per group)
// A workgroup owns a 256-column part of Cin (stage 2: two parts, sharing an XCD as above); every
// part forms the whole dc1 tile (W = 64 / 128 channels: the small tensors are read per part).
// LDS (bytes): W1ᵀ part [256][2W] + dc1 [64][2W] + x [64][512] + dy·bit / dx [64][512]; rows of
// 128 B use the s128 swizzle (row AND transposed reads conflict-free), 512-B rows s512.
template <int WD> struct B1Geom {
  static constexpr int BM = 64, CP = 256;               // pixels per tile, Cin columns per part
  static constexpr int WB = WD * 2;                     // dc1 / W1ᵀ row bytes
  static constexpr int WCPR = WD / 8;                   // 16-byte chunks per dc1 row
  static constexpr int NW = BM * WCPR / 256;            // dc1 chunks per thread per tile
  static constexpr int NX = BM * (CP / 8) / 256;        // x / dy chunks per thread per tile (8)
  static constexpr int W1_BYTES = CP * WB, D_BYTES = BM * WB, X_BYTES = BM * CP * 2;
  static constexpr int LDS = W1_BYTES + D_BYTES + 2 * X_BYTES;
  static constexpr int NWB = WD / 16;                   // dW1 16-row blocks (all waves share)
};

template <int WD> struct B1Raw {
  uint4 d[B1Geom<WD>::NW], c[B1Geom<WD>::NW], x[B1Geom<WD>::NX], y[B1Geom<WD>::NX];
  uint32_t b[B1Geom<WD>::NX];
};

// swizzled byte offset of 16-byte chunk ch of row r in an image with rows of RB bytes
template <int RB>
__device__ __forceinline__ int swz(int r, int ch) {
  if constexpr (RB == 128) return r * 128 + ((ch ^ s128(r & 15)) << 4);
  else return r * RB + ((ch ^ s512(r & 15)) << 4);
}

template <int WD>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1)))
void k_bn1_bwd_dgemm(const uint16_t* __restrict__ da1, const uint16_t* __restrict__ c1,
                     const float* __restrict__ fs, const float* __restrict__ fh,
                     const float* __restrict__ A, const float* __restrict__ B,
                     const float* __restrict__ Cc, const uint16_t* __restrict__ w1t,
                     const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy,
                     const uint8_t* __restrict__ bits, uint16_t* __restrict__ dx,
                     float* __restrict__ slab, int64_t M, int Cin, int tiles, int tpw,
                     int acc_out, int xcd_pairs) {
  using G = B1Geom<WD>;
  constexpr int BM = G::BM, CP = G::CP, WB = G::WB;
  __shared__ __attribute__((aligned(16))) uint8_t lds[G::LDS];
  uint8_t* const sW = lds;                            // W1ᵀ part [CP][WB]
  uint8_t* const sD = lds + G::W1_BYTES;              // dc1      [BM][WB]
  uint8_t* const sX = sD + G::D_BYTES;                // x part   [BM][512]
  uint8_t* const sY = sX + G::X_BYTES;                // dy·bit -> dx [BM][512]
  const int t = threadIdx.x, l = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int g = l >> 4, q = (l & 15) >> 2, p = l & 3;
  const int nparts = Cin / CP;
  const int bx = (int)blockIdx.x & 7, by = (int)blockIdx.x >> 3;
  const int part = xcd_pairs ? by % nparts : (int)blockIdx.x % nparts;
  const int grp = xcd_pairs ? (by / nparts) * 8 + bx : (int)blockIdx.x / nparts;
  const int c0 = part * CP;
  const int u0 = grp * tpw, u1 = min(u0 + tpw, tiles);
  const uint32_t wbytes = (uint32_t)(M * WD * 2), cbytes = (uint32_t)(M * Cin * 2);
  const __amdgpu_buffer_rsrc_t rd = make_rsrc(da1, wbytes), rc = make_rsrc(c1, wbytes);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(x, cbytes), ry = make_rsrc(dy, cbytes);

  // ---- this part's W1ᵀ rows (Cin c0 .. c0 + 255, W contiguous) into LDS (once)
#pragma unroll
  for (int i = 0; i < CP * G::WCPR / 256; ++i) {
    const int e = t + 256 * i, row = e / G::WCPR, ch = e % G::WCPR;
    const uint4 v = *reinterpret_cast<const uint4*>(w1t + (int64_t)(c0 + row) * WD + ch * 8);
    *reinterpret_cast<uint4*>(sW + swz<WB>(row, ch)) = v;
  }
  // ---- apply mapping: dc1 chunk column wc, rows wrow + (256 / WCPR)·i; x / dy: chunk column xc,
  // rows xrow + 8i
  const int wc = t % G::WCPR, wrow = t / G::WCPR;
  const int xc = t & 31, xrow = t >> 5;
  float ca[8], cb[8], ck[8], sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    ca[k] = A[wc * 8 + k]; cb[k] = B[wc * 8 + k]; ck[k] = Cc[wc * 8 + k];
    sc[k] = fs[wc * 8 + k]; sh[k] = fh[wc * 8 + k];
  }

  auto load_tile = [&](int u, B1Raw<WD>& R) {
    const int64_t m0 = (int64_t)u * BM;
#pragma unroll
    for (int i = 0; i < G::NW; ++i) {
      const int64_t m = m0 + wrow + (256 / G::WCPR) * i;
      const uint32_t off = m < M ? (uint32_t)((m * WD + wc * 8) * 2) : OOB;
      R.d[i] = bload16(rd, off);
      R.c[i] = bload16(rc, off);
    }
#pragma unroll
    for (int i = 0; i < G::NX; ++i) {
      const int64_t m = m0 + xrow + 8 * i;
      const uint32_t off = m < M ? (uint32_t)((m * Cin + c0 + xc * 8) * 2) : OOB;
      R.x[i] = bload16(rx, off);
      R.y[i] = bload16(ry, off);
      R.b[i] = m < M ? (uint32_t)bits[(m * Cin + c0) / 8 + xc] : 0u;
    }
  };

  f32x4 acc2[G::NWB][4];                 // dW1 rows 16i.., Cin columns 64w + 16j ..
#pragma unroll
  for (int i = 0; i < G::NWB; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto phase_a = [&](const B1Raw<WD>& R) {
#pragma unroll
    for (int i = 0; i < G::NW; ++i) {
      const uint32_t dw[4] = {R.d[i].x, R.d[i].y, R.d[i].z, R.d[i].w};
      const uint32_t cw[4] = {R.c[i].x, R.c[i].y, R.c[i].z, R.c[i].w};
      uint32_t o[4];
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2) {
        const float x0 = hlo(cw[k2]), x1 = hhi(cw[k2]);
        float d0 = hlo(dw[k2]), d1 = hhi(dw[k2]);
        d0 = fmaf(x0, sc[2 * k2], sh[2 * k2]) > 0.f ? d0 : 0.f;
        d1 = fmaf(x1, sc[2 * k2 + 1], sh[2 * k2 + 1]) > 0.f ? d1 : 0.f;
        const float v0 = ca[2 * k2] * d0 + cb[2 * k2] * x0 + ck[2 * k2];
        const float v1 = ca[2 * k2 + 1] * d1 + cb[2 * k2 + 1] * x1 + ck[2 * k2 + 1];
        o[k2] = (uint32_t)f2h(v0) | ((uint32_t)f2h(v1) << 16);
      }
      const int row = wrow + (256 / G::WCPR) * i;
      *reinterpret_cast<uint4*>(sD + swz<WB>(row, wc)) = make_uint4(o[0], o[1], o[2], o[3]);
    }
#pragma unroll
    for (int i = 0; i < G::NX; ++i) {
      const int row = xrow + 8 * i;
      *reinterpret_cast<uint4*>(sX + swz<512>(row, xc)) = R.x[i];
      // the masked addend dy·bit, rounded like the GEMM epilogue's addend (bf16 in, fp32 add)
      *reinterpret_cast<uint4*>(sY + swz<512>(row, xc)) = mask_h16x8(R.y[i], R.b[i]);
    }
  };

  auto phase_b = [&](int u) {
    // dW1[w][cin] += dc1ᵀ[w][px] · x[px][cin], K = 64 pixels: wave w takes Cin columns 64w..
#pragma unroll
    for (int kk = 0; kk < BM / 32; ++kk) {
      i16x4 ta[2][G::NWB], tb[2][4];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int px = 32 * kk + 8 * g + q + 4 * hh;
#pragma unroll
        for (int i = 0; i < G::NWB; ++i)
          ta[hh][i] = tr_read(sD + swz<WB>(px, 2 * i + (p >> 1)) + 8 * (p & 1));
#pragma unroll
        for (int j = 0; j < 4; ++j)
          tb[hh][j] = tr_read(sX + swz<512>(px, 2 * (4 * w + j) + (p >> 1)) + 8 * (p & 1));
      }
      h16x8 fb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = cat8(tb[0][j], tb[1][j]);
#pragma unroll
      for (int i = 0; i < G::NWB; ++i) {
        const h16x8 fa = cat8(ta[0][i], ta[1][i]);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc2[i][j] = mfma16(fa, fb[j], acc2[i][j]);
      }
    }
    // dx tile: D[cin 64w + 16j ..][px] = W1ᵀ[cin][w] · dc1[px][w]ᵀ, K = W
    f32x4 acc1[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc1[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < WD / 32; ++ks) {
      const int ch = 4 * ks + g;
      h16x8 fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        fb[i] = *reinterpret_cast<const h16x8*>(sD + swz<WB>(16 * i + (l & 15), ch));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const h16x8 fa = *reinterpret_cast<const h16x8*>(sW + swz<WB>(64 * w + 16 * j + (l & 15), ch));
#pragma unroll
        for (int i = 0; i < 4; ++i) acc1[j][i] = mfma16(fa, fb[i], acc1[j][i]);
      }
    }
    // epilogue: lane holds cin 64w + 16j + 4g .. +3 of pixel 16i + (l & 15); dx = round(acc)
    // + addend (the GEMM epilogue's order: bf16(acc) then + addend, rounded again)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int px = 16 * i + (l & 15);
        const int cin = 64 * w + 16 * j + 4 * g;
        uint2* ptr = reinterpret_cast<uint2*>(sY + swz<512>(px, cin >> 3) + 8 * ((cin >> 2) & 1));
        const uint2 a = *ptr;
        const float s0 = h2f(f2h(acc1[j][i][0])) + hlo(a.x), s1 = h2f(f2h(acc1[j][i][1])) + hhi(a.x);
        const float s2 = h2f(f2h(acc1[j][i][2])) + hlo(a.y), s3 = h2f(f2h(acc1[j][i][3])) + hhi(a.y);
        *ptr = make_uint2((uint32_t)f2h(s0) | ((uint32_t)f2h(s1) << 16),
                          (uint32_t)f2h(s2) | ((uint32_t)f2h(s3) << 16));
      }
    __syncthreads();
    const int64_t m0 = (int64_t)u * BM;
#pragma unroll
    for (int i = 0; i < G::NX; ++i) {
      const int row = xrow + 8 * i;
      if (m0 + row < M)
        *reinterpret_cast<uint4*>(dx + (m0 + row) * Cin + c0 + xc * 8) =
            *reinterpret_cast<const uint4*>(sY + swz<512>(row, xc));
    }
  };

  B1Raw<WD> R0;
  if (u0 < u1) load_tile(u0, R0);
  for (int u = u0; u < u1; ++u) {
    phase_a(R0);
    __syncthreads();
    if (u + 1 < u1) load_tile(u + 1, R0);
    phase_b(u);
    __syncthreads();                     // dx staging read before the next tile overwrites it
  }
  // ---- slab: lane holds D[w = 16i + 4g + r][cin = c0 + 64w + 16j + (l & 15)]
  float* sl = slab + (int64_t)grp * WD * Cin;
#pragma unroll
  for (int i = 0; i < G::NWB; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float* d = sl + (int64_t)(16 * i + 4 * g + r) * Cin + c0 + 64 * w + 16 * j + (l & 15);
        *d = acc_out ? *d + acc2[i][j][r] : acc2[i][j][r];
      }
}

bool bn1_bwd_dgemm_ok(int64_t M, int Wd, int Cin) {
  return ((Wd == 64 && Cin == 256) || (Wd == 128 && Cin == 512)) && M > 0 &&
         M * Cin * 2 < (int64_t(1) << 31);
}

int bn1_bwd_dgemm_slabs(int64_t M, int Wd, int Cin) {
  const int tiles = (int)((M + 63) / 64), nparts = Cin / 256;
  const int want = std::max(8, cu_count() / nparts / 8 * 8);
  const int tpw = (tiles + want - 1) / want;
  const int used = (tiles + tpw - 1) / tpw;
  return used <= 1 ? 1 : (used + 7) / 8 * 8;
}

void bn1_bwd_dgemm(const uint16_t* da1, const uint16_t* c1, const float* fs, const float* fh,
                   const float* A, const float* B, const float* Cc, const uint16_t* w1t,
                   const uint16_t* x, const uint16_t* dy, const uint8_t* bits, uint16_t* dx,
                   float* slab, int64_t M, int Wd, int Cin, bool acc_out, hipStream_t st) {
  const int tiles = (int)((M + 63) / 64), nparts = Cin / 256;
  const int groups = bn1_bwd_dgemm_slabs(M, Wd, Cin);
  const int tpw = (tiles + groups - 1) / groups;
  const int acc = (acc_out && groups == 1) ? 1 : 0;
  const int blocks = groups * nparts, xp = groups % 8 == 0 ? 1 : 0;
  if (Wd == 64)
    hipLaunchKernelGGL(k_bn1_bwd_dgemm<64>, dim3(blocks), dim3(256), 0, st, da1, c1, fs, fh, A, B,
                       Cc, w1t, x, dy, bits, dx, slab, M, Cin, tiles, tpw, acc, xp);
  else
    hipLaunchKernelGGL(k_bn1_bwd_dgemm<128>, dim3(blocks), dim3(256), 0, st, da1, c1, fs, fh, A,
                       B, Cc, w1t, x, dy, bits, dx, slab, M, Cin, tiles, tpw, acc, xp);
}

}  // namespace lw
