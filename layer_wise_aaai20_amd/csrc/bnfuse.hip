// BatchNorm-backward apply fused with BOTH GEMMs that consume its output, for the ResNet-50
// stage-1 bottleneck's BN3 (C = 256 channels of c3, 64 of a2), gfx950.
//
// The per-layer path (ops/block.py) runs, after BN3's reduce + finalize:
//   dc3 = A·(dr·bit) + B·c3 + C          k_bn_bwd_apply  reads dr, c3, bits; writes dc3 (256 ch)
//   dW3 += dc3ᵀ · a2                     GEMM            reads dc3 again (+ a2)
//   da2  = dc3 · W3                      GEMM            reads dc3 a third time, writes da2
// i.e. five 256-channel activation streams (411 MB each at batch 256, 56x56). Here one persistent
// kernel reads dr, c3 and the bitmap ONCE per 64-pixel tile, forms the bf16 dc3 tile in LDS (the
// apply's exact expression and rounding) and feeds both products from that LDS image:
//   da2 tile [64 px][64]   = dc3 tile · W3       (W3ᵀ resident in LDS, K = 256 channels)
//   dW3 [256][64]         += dc3 tileᵀ · a2 tile (accumulated in registers across the tiles of the
//                                                 workgroup, K = pixels; one fp32 slab per
//                                                 workgroup, summed in fixed order by the split-K
//                                                 reduce, gemm.hip)
// -> two 256-channel streams instead of five (profiles/r6: 230 + 117 + 91 us per block before).
//
// LDS images (bf16, 16-byte chunks XOR-swizzled by row so that every fragment read is
// bank-conflict-free; scripts/probes check in the tests):
//   W3ᵀ [64 ci][256 co] and dc3 [64 px][256 co]: 512-B rows, chunk c at c ^ s512(row), read by
//     rows with ds_read_b128 (16 rows x chunks 2k, 2k+1 per 16-lane group: s512 distinct) and, for
//     dc3, by columns with ds_read_b64_tr_b16 (the A operand dc3ᵀ of dW3);
//   a2 [64 px][64 ci]: 128-B rows, chunk c at c ^ s128(row), read by columns (B operand of dW3);
//   da2 staging [64 px][64 ci] for 16-byte global stores.
// Waves (4, 256 threads, two workgroups per CU): da2 rows 16w..16w+15 of ci x 64 px (4 MFMA
// blocks); dW3 co 64w..64w+63 x all 64 ci (16 MFMA blocks). Per tile and wave: 32 + 32 MFMAs.
#include "gemm_core.h"

#include <cstdlib>

namespace lw {

namespace {
constexpr int BF_BM = 64;                 // pixels per tile
constexpr int BF_CO = 256, BF_CI = 64;
constexpr int BF_LDS = 32768 + 32768 + 8192 + 8192;

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
}  // namespace

template <int OCC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC)))
void k_bn3_bwd_dgemm(const uint16_t* __restrict__ dr, const uint16_t* __restrict__ c3,
                     const uint8_t* __restrict__ bits, const float* __restrict__ A,
                     const float* __restrict__ B, const float* __restrict__ Cc,
                     const uint16_t* __restrict__ w3t, const uint16_t* __restrict__ a2,
                     uint16_t* __restrict__ da2, float* __restrict__ slab, int64_t M, int tiles,
                     int tpw) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[BF_LDS];
  uint8_t* const sW = lds;                 // W3ᵀ  [64][512 B]
  uint8_t* const sD = lds + 32768;         // dc3  [64][512 B]
  uint8_t* const sA = lds + 65536;         // a2   [64][128 B]
  uint8_t* const sO = lds + 73728;         // da2  [64][128 B]
  const int t = threadIdx.x, l = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int g = l >> 4, q = (l & 15) >> 2, p = l & 3;
  const int u0 = (int)blockIdx.x * tpw, u1 = min(u0 + tpw, tiles);
  const uint32_t act_bytes = (uint32_t)(M * BF_CO * 2), a2_bytes = (uint32_t)(M * BF_CI * 2);
  const __amdgpu_buffer_rsrc_t rdr = make_rsrc(dr, act_bytes), rc3 = make_rsrc(c3, act_bytes);
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(a2, a2_bytes);

  // ---- W3ᵀ into LDS (once)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int e = t + 256 * i, row = e >> 5, ch = e & 31;
    const uint4 v = *reinterpret_cast<const uint4*>(w3t + row * BF_CO + ch * 8);
    *reinterpret_cast<uint4*>(sW + row * 512 + ((ch ^ s512(row & 15)) << 4)) = v;
  }
  // ---- this thread's 8 channels of the apply: chunk column cc, rows t/32 + 8i
  const int cc = t & 31, prow = t >> 5;
  float ca[8], cb[8], ck[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { ca[k] = A[cc * 8 + k]; cb[k] = B[cc * 8 + k]; ck[k] = Cc[cc * 8 + k]; }

  uint4 vd[8], vx[8], va[2];
  uint32_t vb[8];
  auto load_tile = [&](int u) {
    const int64_t m0 = (int64_t)u * BF_BM;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t m = m0 + prow + 8 * i;
      const uint32_t off = m < M ? (uint32_t)((m * BF_CO + cc * 8) * 2) : OOB;
      vd[i] = bload16(rdr, off);
      vx[i] = bload16(rc3, off);
      vb[i] = m < M ? (uint32_t)bits[m * (BF_CO / 8) + cc] : 0u;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = t + 256 * i;
      const int64_t m = m0 + (e >> 3);
      va[i] = bload16(ra, m < M ? (uint32_t)((m * BF_CI + (e & 7) * 8) * 2) : OOB);
    }
  };

  f32x4 acc2[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (u0 < u1) load_tile(u0);
  for (int u = u0; u < u1; ++u) {
    // ---- phase A: dc3 = A·(dr·bit) + B·c3 + C (bf16) and a2 into their LDS images
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t dw[4] = {vd[i].x, vd[i].y, vd[i].z, vd[i].w};
      const uint32_t xw[4] = {vx[i].x, vx[i].y, vx[i].z, vx[i].w};
      uint32_t o[4];
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2) {
        float d0 = hlo(dw[k2]), d1 = hhi(dw[k2]);
        d0 = ((vb[i] >> (2 * k2)) & 1u) ? d0 : 0.f;
        d1 = ((vb[i] >> (2 * k2 + 1)) & 1u) ? d1 : 0.f;
        const float o0 = ca[2 * k2] * d0 + cb[2 * k2] * hlo(xw[k2]) + ck[2 * k2];
        const float o1 = ca[2 * k2 + 1] * d1 + cb[2 * k2 + 1] * hhi(xw[k2]) + ck[2 * k2 + 1];
        o[k2] = (uint32_t)f2h(o0) | ((uint32_t)f2h(o1) << 16);
      }
      const int row = prow + 8 * i;
      *reinterpret_cast<uint4*>(sD + row * 512 + ((cc ^ s512(row & 15)) << 4)) =
          make_uint4(o[0], o[1], o[2], o[3]);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = t + 256 * i, row = e >> 3, ch = e & 7;
      *reinterpret_cast<uint4*>(sA + row * 128 + ((ch ^ s128(row & 15)) << 4)) = va[i];
    }
    __syncthreads();
    if (u + 1 < u1) load_tile(u + 1);      // in flight under this tile's MFMAs

    // ---- da2 tile: D[ci 16w..][px] = W3ᵀ[ci][co] · dc3[px][co]ᵀ, K = 256 channels
    f32x4 acc1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc1[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int ci_r = 16 * w + (l & 15);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int ch = 4 * ks + g;
      const h16x8 fa = *reinterpret_cast<const h16x8*>(sW + ci_r * 512 + ((ch ^ s512(ci_r & 15)) << 4));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int px = 16 * j + (l & 15);
        const h16x8 fb = *reinterpret_cast<const h16x8*>(sD + px * 512 + ((ch ^ s512(px & 15)) << 4));
        acc1[j] = mfma16(fa, fb, acc1[j]);
      }
    }
    // ---- dW3[co 64w..][ci] += dc3ᵀ[co][px] · a2[px][ci], K = 64 pixels (transposing reads)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      i16x4 ta[2][4], tb[2][4];           // [rows 8g+q / 8g+4+q][block]
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int px = 32 * kk + 8 * g + q + 4 * hh;
        const uint8_t* rowD = sD + px * 512;
        const uint8_t* rowA = sA + px * 128;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int chd = 2 * (4 * w + i) + (p >> 1);
          ta[hh][i] = tr_read(rowD + ((chd ^ s512(px & 15)) << 4) + 8 * (p & 1));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int cha = 2 * j + (p >> 1);
          tb[hh][j] = tr_read(rowA + ((cha ^ s128(px & 15)) << 4) + 8 * (p & 1));
        }
      }
      h16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) { fa[i] = cat8(ta[0][i], ta[1][i]); fb[i] = cat8(tb[0][i], tb[1][i]); }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc2[i][j] = mfma16(fa[i], fb[j], acc2[i][j]);
    }
    // ---- da2 tile -> staging (lane: ci 16w + 4g .. +3 of pixel 16j + (l & 15))
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int px = 16 * j + (l & 15);
      const int ch = 2 * w + (g >> 1);
      uint16_t h[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) h[r] = f2h(acc1[j][r]);
      *reinterpret_cast<uint2*>(sO + px * 128 + ((ch ^ s128(px & 15)) << 4) + 8 * (g & 1)) =
          make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16));
    }
    __syncthreads();
    const int64_t m0 = (int64_t)u * BF_BM;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = t + 256 * i, row = e >> 3, ch = e & 7;
      if (m0 + row < M)
        *reinterpret_cast<uint4*>(da2 + (m0 + row) * BF_CI + ch * 8) =
            *reinterpret_cast<const uint4*>(sO + row * 128 + ((ch ^ s128(row & 15)) << 4));
    }
  }
  // ---- this workgroup's dW3 slab: lane holds D[co = 64w + 16i + 4g + r][ci = 16j + (l & 15)]
  float* sl = slab + (int64_t)blockIdx.x * BF_CO * BF_CI;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        sl[(64 * w + 16 * i + 4 * g + r) * BF_CI + 16 * j + (l & 15)] = acc2[i][j][r];
}

// workgroups per CU: 1 (512 VGPRs, no spill) or 2 (256 VGPRs: 72 bytes of scratch) —
// LWAAAI_BN3_OCC, default measured
static int bf_occ() {
  static const int occ = [] {
    const char* e = std::getenv("LWAAAI_BN3_OCC");
    return (e && e[0] == '2') ? 2 : 1;
  }();
  return occ;
}

int bn3_bwd_dgemm_blocks(int64_t M) {
  const int64_t tiles = (M + BF_BM - 1) / BF_BM;
  const int64_t want = bf_occ() * (int64_t)cu_count();
  const int64_t tpw = (tiles + want - 1) / want;
  return (int)((tiles + tpw - 1) / tpw);
}

bool bn3_bwd_dgemm_ok(int64_t M, int C, int Ci) {
  return C == BF_CO && Ci == BF_CI && M > 0 && M * BF_CO * 2 < (int64_t(1) << 31);
}

void bn3_bwd_dgemm(const uint16_t* dr, const uint16_t* c3, const uint8_t* bits, const float* A,
                   const float* B, const float* Cc, const uint16_t* w3t, const uint16_t* a2,
                   uint16_t* da2, float* slab, int64_t M, hipStream_t st) {
  const int64_t tiles = (M + BF_BM - 1) / BF_BM;
  const int blocks = bn3_bwd_dgemm_blocks(M);
  const int tpw = (int)((tiles + blocks - 1) / blocks);
  if (bf_occ() == 2)
    hipLaunchKernelGGL(k_bn3_bwd_dgemm<2>, dim3(blocks), dim3(256), 0, st, dr, c3, bits, A, B, Cc,
                       w3t, a2, da2, slab, M, (int)tiles, tpw);
  else
    hipLaunchKernelGGL(k_bn3_bwd_dgemm<1>, dim3(blocks), dim3(256), 0, st, dr, c3, bits, A, B, Cc,
                       w3t, a2, da2, slab, M, (int)tiles, tpw);
}

}  // namespace lw
