// ResNet stem backward, fused: the BatchNorm + ReLU + 3x3/2 max-pool backward apply and the 7x7/2
// convolution's weight gradient in one persistent kernel (gfx950).
//
// The per-layer path (ops/nn.py _StemConvPoolFn) runs, after the pooled-side statistics pass:
//   dc = A·(routed pooled gradient, ReLU-masked) + B·c + C    k_stem_pool_bwd_s2: reads dp, the
//                                                              window-slot bytes and c (the 112x112
//                                                              conv output); writes dc (411 MB at
//                                                              batch 256)
//   dW = dcᵀ · im2col(x)                                       implicit-GEMM weight gradient:
//                                                              reads dc again + the image
// (profiles/r6: 218 + 234 us). Here a workgroup walks the pooled rows of one image range: per
// pooled row it forms the 224-pixel dc tile (two conv rows) in LDS exactly as the apply kernel
// does, stages the 9-row x 232-pixel window of the 4-channel image that those rows' 7x7/2 windows
// read, and accumulates dW[64][7 x 8 x 4] with v_mfma_f32_16x16x32 — the pixel index is K, both
// operands read with ds_read_b64_tr_b16 (the image operand's lane addresses are the im2col gather
// itself: 4 channels = one 8-byte pixel). dc never reaches memory; fp32 slabs per workgroup are
// summed by the split-K reduce (gemm.hip). The dW column layout [co][r][s 0..7][ci 0..3] is the
// implicit GEMM's for a 4-channel image (tap s = 7 and channel 3 are padding, dropped by the
// caller).
#include "gemm_core.h"

namespace lw {

namespace {
constexpr int SF_C = 64;                      // conv output channels
constexpr int SF_W = 112, SF_PX = 2 * SF_W;   // conv output width, pixels per tile (two rows)
constexpr int SF_PW = 232;                    // patch row: input columns -4 .. 227
constexpr int SF_PR = 9;                      // patch rows: 4yo - 3 .. 4yo + 5
constexpr int SF_N = 224;                     // dW columns: 7 rows x 8 taps x 4 channels
constexpr int SF_DC_BYTES = SF_PX * 128;      // dc tile [224][64] bf16
constexpr int SF_X_BYTES = SF_PR * SF_PW * 8;
constexpr int SF_ITEMS = (SF_W / 2) * (SF_C / 8);          // 2x2 blocks x channel groups = 448
constexpr int SF_XCH = SF_PR * SF_PW / 2;                  // 16-byte patch chunks = 1044
constexpr int SF_XPT = (SF_XCH + 255) / 256;               // per thread (5)

__device__ __forceinline__ int sf_s128(int r) { return (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2); }
__device__ __forceinline__ int sf_dc(int px, int ch) { return px * 128 + ((ch ^ sf_s128(px & 15)) << 4); }

typedef __attribute__((address_space(3))) i16x4 sf_lds_v4;
__device__ __forceinline__ i16x4 sf_tr(const uint8_t* a) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((sf_lds_v4*)a);
}
__device__ __forceinline__ h16x8 sf_cat8(i16x4 lo, i16x4 hi) {
  typedef short i16x8 __attribute__((ext_vector_type(8)));
  const i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(h16x8, v);
}

struct SfRaw {
  uint4 d[2][2][2];       // [item][u][v] pooled gradient (8 channels)
  uint2 s[2][2][2];       // [item][u][v] window-slot bytes
  uint4 c[2][2][2];       // [item][ay][bx] conv output
  uint4 x[SF_XPT];        // image patch chunks
};
}  // namespace

// One workgroup per CU; tile t = (image n, pooled row yo) for t in [t0, t1).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1)))
void k_stem_bwd_wgrad(const uint16_t* __restrict__ dp, const uint8_t* __restrict__ idx,
                      const uint16_t* __restrict__ c, const float* __restrict__ scale,
                      const float* __restrict__ shift, const float* __restrict__ A,
                      const float* __restrict__ B, const float* __restrict__ Cc,
                      const uint16_t* __restrict__ x4, float* __restrict__ slab, int N, int Ho,
                      int Wo, int Hin, int Win, int tpw) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[SF_DC_BYTES + SF_X_BYTES];
  uint8_t* const sD = lds;
  uint8_t* const sX = lds + SF_DC_BYTES;
  const int t = threadIdx.x, l = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int g = l >> 4, q = (l & 15) >> 2, p = l & 3;
  const int tiles = N * Ho;
  const int t0 = (int)blockIdx.x * tpw, t1 = min(t0 + tpw, tiles);
  const int H = 2 * Ho;                                   // conv output height (= 2 Ho)
  const int cg = t & 7;                                   // this thread's 8 channels (fixed)
  float sc[8], sh[8], ca[8], cb[8], ck[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = scale[cg * 8 + j]; sh[j] = shift[cg * 8 + j];
    ca[j] = A[cg * 8 + j]; cb[j] = B[cg * 8 + j]; ck[j] = Cc[cg * 8 + j];
  }
  const uint32_t x_bytes = (uint32_t)((int64_t)N * Hin * Win * 8);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(x4, x_bytes);

  auto load_tile = [&](int tt, SfRaw& R) {
    const int n = tt / Ho, yo = tt - n * Ho;
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int e = t + 256 * it;
      const bool on = e < SF_ITEMS;
      const int xo = e >> 3;
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v) {
          const bool in = on && yo + u < Ho && xo + v < Wo;
          const int64_t o = (((int64_t)n * Ho + yo + u) * Wo + xo + v) * SF_C + cg * 8;
          R.d[it][u][v] = in ? *reinterpret_cast<const uint4*>(dp + o) : make_uint4(0u, 0u, 0u, 0u);
          R.s[it][u][v] = in ? *reinterpret_cast<const uint2*>(idx + o)
                             : make_uint2(0xffffffffu, 0xffffffffu);   // slot 255 matches nothing
        }
#pragma unroll
      for (int ay = 0; ay < 2; ++ay)
#pragma unroll
        for (int bx = 0; bx < 2; ++bx)
          R.c[it][ay][bx] = on ? *reinterpret_cast<const uint4*>(
                                     c + (((int64_t)n * H + 2 * yo + ay) * SF_W + 2 * xo + bx) * SF_C + cg * 8)
                               : make_uint4(0u, 0u, 0u, 0u);
    }
    // image patch: rows 4yo - 3 .. 4yo + 5, columns -4 .. 227 (two pixels per 16-byte chunk;
    // outside the image: zeros through the buffer range check)
#pragma unroll
    for (int i = 0; i < SF_XPT; ++i) {
      const int e = t + 256 * i;
      const int pr = e / (SF_PW / 2), pc = (e - pr * (SF_PW / 2)) * 2;
      const int iy = 4 * yo - 3 + pr, ix = pc - 4;
      const bool ok = e < SF_XCH && iy >= 0 && iy < Hin && ix >= 0 && ix < Win;
      R.x[i] = bload16(rx, ok ? (uint32_t)((((int64_t)n * Hin + iy) * Win + ix) * 8) : OOB);
    }
  };

  f32x4 acc[2][7];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 7; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- phase A: dc of the tile's 2x2 blocks (k_stem_pool_bwd_s2's routing, mask and apply)
  auto phase_a = [&](const SfRaw& R) {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int e = t + 256 * it;
      if (e < SF_ITEMS) {
        const int xo = e >> 3;
        float d[2][2][8];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int v = 0; v < 2; ++v) {
            const uint32_t wd[4] = {R.d[it][u][v].x, R.d[it][u][v].y, R.d[it][u][v].z, R.d[it][u][v].w};
#pragma unroll
            for (int k = 0; k < 4; ++k) { d[u][v][2 * k] = hlo(wd[k]); d[u][v][2 * k + 1] = hhi(wd[k]); }
          }
#pragma unroll
        for (int ay = 0; ay < 2; ++ay)
#pragma unroll
          for (int bx = 0; bx < 2; ++bx) {
            const uint32_t wc[4] = {R.c[it][ay][bx].x, R.c[it][ay][bx].y, R.c[it][ay][bx].z, R.c[it][ay][bx].w};
            uint32_t o[4];
#pragma unroll
            for (int k2 = 0; k2 < 4; ++k2) {
              float ov[2];
#pragma unroll
              for (int h = 0; h < 2; ++h) {
                const int j = 2 * k2 + h;
                float a = 0.f;
#pragma unroll
                for (int u = 0; u <= ay; ++u)
#pragma unroll
                  for (int v = 0; v <= bx; ++v) {
                    const int kh = 1 + ay - 2 * u, kw = 1 + bx - 2 * v;
                    const uint32_t ws = j < 4 ? R.s[it][u][v].x : R.s[it][u][v].y;
                    const int slot = (int)((ws >> (8 * (j & 3))) & 0xffu);
                    a += slot == kh * 3 + kw ? d[u][v][j] : 0.f;
                  }
                const float xv = h ? hhi(wc[k2]) : hlo(wc[k2]);
                const float dz = fmaf(xv, sc[j], sh[j]) > 0.f ? a : 0.f;
                ov[h] = ca[j] * dz + cb[j] * xv + ck[j];
              }
              o[k2] = (uint32_t)f2h(ov[0]) | ((uint32_t)f2h(ov[1]) << 16);
            }
            *reinterpret_cast<uint4*>(sD + sf_dc(ay * SF_W + 2 * xo + bx, cg)) =
                make_uint4(o[0], o[1], o[2], o[3]);
          }
      }
    }
#pragma unroll
    for (int i = 0; i < SF_XPT; ++i) {
      const int e = t + 256 * i;
      if (e < SF_XCH) *reinterpret_cast<uint4*>(sX + e * 16) = R.x[i];
    }
  };

  // ---- phase B: dW[co][n] += dcᵀ[co][px] · im2col[px][n]; wave w: co blocks 2(w&1), +1 and
  // n blocks 7(w>>1) .. +6; K = the tile's 224 pixels
  const int cb0 = 2 * (w & 1), nb0 = 7 * (w >> 1);
  auto phase_b = [&]() {
#pragma unroll 1
    for (int kk = 0; kk < SF_PX / 32; ++kk) {
      i16x4 ta[2][2], tb[2][7];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int k = 32 * kk + 8 * g + q + 4 * hh;       // pixel of the tile (this lane's row)
        const int ay = k >= SF_W ? 1 : 0, xx = k - ay * SF_W;
#pragma unroll
        for (int i = 0; i < 2; ++i)
          ta[hh][i] = sf_tr(sD + sf_dc(k, 2 * (cb0 + i) + (p >> 1)) + 8 * (p & 1));
#pragma unroll
        for (int j = 0; j < 7; ++j) {
          const int nb = nb0 + j, r = nb >> 1, s = 4 * (nb & 1) + p;
          tb[hh][j] = sf_tr(sX + ((2 * ay + r) * SF_PW + 2 * xx + 1 + s) * 8);
        }
      }
      h16x8 fa[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = sf_cat8(ta[0][i], ta[1][i]);
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        const h16x8 fb = sf_cat8(tb[0][j], tb[1][j]);
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][j] = mfma16(fa[i], fb, acc[i][j]);
      }
    }
  };

  SfRaw R0;
  if (t0 < t1) load_tile(t0, R0);
  for (int tt = t0; tt < t1; ++tt) {
    phase_a(R0);
    __syncthreads();
    if (tt + 1 < t1) load_tile(tt + 1, R0);
    phase_b();
    __syncthreads();
  }
  // ---- slab: lane holds D[co = 16(cb0 + i) + 4g + r][n = 16(nb0 + j) + (l & 15)]
  float* sl = slab + (int64_t)blockIdx.x * SF_C * SF_N;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 7; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        sl[(16 * (cb0 + i) + 4 * g + r) * SF_N + 16 * (nb0 + j) + (l & 15)] = acc[i][j][r];
}

bool stem_bwd_wgrad_ok(int C, int H, int W, int Ho, int Wo, int Hin, int Win) {
  return C == SF_C && W == SF_W && H == 2 * Ho && W == 2 * Wo && Hin == 2 * H && Win == 2 * W;
}

int stem_bwd_wgrad_blocks(int N, int Ho) {
  const int tiles = N * Ho, cus = cu_count();
  const int tpw = (tiles + cus - 1) / cus;
  return (tiles + tpw - 1) / tpw;
}

void stem_bwd_wgrad(const uint16_t* dp, const uint8_t* idx, const uint16_t* c, const float* scale,
                    const float* shift, const float* A, const float* B, const float* Cc,
                    const uint16_t* x4, float* slab, int N, int Ho, int Wo, int Hin, int Win,
                    hipStream_t st) {
  const int tiles = N * Ho;
  const int blocks = stem_bwd_wgrad_blocks(N, Ho);
  const int tpw = (tiles + blocks - 1) / blocks;
  hipLaunchKernelGGL(k_stem_bwd_wgrad, dim3(blocks), dim3(256), 0, st, dp, idx, c, scale, shift,
                     A, B, Cc, x4, slab, N, Ho, Wo, Hin, Win, tpw);
}

}  // namespace lw
