// Implicit-GEMM convolutions for gfx950: forward, data gradient and weight gradient of NHWC bf16
// convolutions on the MFMA GEMM core of gemm_core.h.
//
// No im2col buffer is ever written: the GEMM operand that is a convolution window is gathered
// straight from the activation tensor while a K-step is staged into LDS (gemm_core.h
// load_tile_gather_a / load_tile_gather_b), with the zero padding produced by the bounds test.
// Everything else — MFMA main loop, double-buffered LDS, XCD-aware tile order, BN-apply+ReLU
// prologue, column-statistics / split-K / fp32-accumulate epilogues — is the plain GEMM's.
//
//   forward   rows = output pixels, k = (r, s, ci): y = im2col(x)·Wᵀ       W = [Co][R][S][C]
//             (a channels_last conv weight is already that matrix). The BatchNorm-apply+ReLU of
//             the input runs in the staging prologue (channel = ci), so a bottleneck's
//             relu(bn1(c1)) is never materialised, and the epilogue can emit the next BN's
//             column statistics.
//   dgrad     rows = input pixels, k = (tap, co): dx = im2col'(dy)·Wt     Wt = [tap][Co][C]
//             with the taps walked backwards (dh = dw = -1). A stride-2 convolution splits into
//             its 4 output-parity classes (blockIdx.z), each a dense stride-1 problem over only
//             the taps that reach it — no multiply by structural zeros — whose rows are scattered
//             back to their pixels by the epilogue's row map.
//   wgrad     dW[co][(r, s, ci)] = Σ_pix dy[pix][co] · im2col(x)[pix][(r, s, ci)]; the reduction
//             over N·Ho·Wo pixels is split over workgroups (fixed-order slab reduce) and the fp32
//             result is accumulated straight into the gradient arena.
//   C == 4    (a 3-channel image padded to 4): the 16-byte chunk is two horizontally adjacent
//             taps of one pixel pair, so the stem conv runs on the same kernel.
#include "gemm_core.h"

namespace lw {

// K-contiguous data-gradient weight pack, one launch: out[i][c][k] for parity class i,
// k = (jr * TS + js) * Co + o < TR * TS * Co, = w[o][r0 + sh * jr][s0 + sw * js][c] (channels_last
// [Co][R][S][C] source), zero up to the row stride kmax. Each thread writes 8 consecutive k (one
// 16-byte store); the gathered reads hit L2 (a weight is at most a few MB). A 1x1 convolution
// (one class, R = S = 1) is the plain transpose Wᵀ.
struct PackClasses { int r0[4], s0[4], TR[4], TS[4]; };

__global__ __launch_bounds__(256) void k_pack_dgrad_kc(const uint16_t* __restrict__ w,
                                                       uint16_t* __restrict__ out, int Co, int C,
                                                       int R, int S, int sh, int sw, int nclass,
                                                       PackClasses pc, int kmax) {
  const int64_t per_row = kmax / 8, per_class = (int64_t)C * per_row;
  const int64_t total = nclass * per_class;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * 256) {
    const int i = (int)(t / per_class);
    const int64_t rem = t - i * per_class;
    const int c = (int)(rem / per_row);
    const int k0 = (int)(rem - (int64_t)c * per_row) * 8;
    const int r0 = i == 0 ? pc.r0[0] : i == 1 ? pc.r0[1] : i == 2 ? pc.r0[2] : pc.r0[3];
    const int s0 = i == 0 ? pc.s0[0] : i == 1 ? pc.s0[1] : i == 2 ? pc.s0[2] : pc.s0[3];
    const int TR = i == 0 ? pc.TR[0] : i == 1 ? pc.TR[1] : i == 2 ? pc.TR[2] : pc.TR[3];
    const int TS = i == 0 ? pc.TS[0] : i == 1 ? pc.TS[1] : i == 2 ? pc.TS[2] : pc.TS[3];
    const int Kc = TR * TS * Co;
    uint16_t v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k = k0 + q;
      uint16_t x = 0;
      if (k < Kc) {
        const int tap = k / Co, o = k - tap * Co;
        const int jr = tap / TS, js = tap - jr * TS;
        const int r = r0 + sh * jr, sx = s0 + sw * js;
        x = w[(((int64_t)o * R + r) * S + sx) * C + c];
      }
      v[q] = x;
    }
    *reinterpret_cast<uint4*>(out + (int64_t)i * C * kmax + (int64_t)c * kmax + k0) =
        make_uint4((uint32_t)v[0] | ((uint32_t)v[1] << 16), (uint32_t)v[2] | ((uint32_t)v[3] << 16),
                   (uint32_t)v[4] | ((uint32_t)v[5] << 16), (uint32_t)v[6] | ((uint32_t)v[7] << 16));
  }
}

void pack_dgrad_kc(const uint16_t* w, uint16_t* out, int Co, int C, int R, int S, int sh, int sw,
                   int nclass, const int* r0, const int* s0, const int* TR, const int* TS,
                   int kmax, hipStream_t st) {
  PackClasses pc{};
  for (int i = 0; i < nclass; ++i) {
    pc.r0[i] = r0[i]; pc.s0[i] = s0[i]; pc.TR[i] = TR[i]; pc.TS[i] = TS[i];
  }
  const int64_t total = (int64_t)nclass * C * (kmax / 8);
  int64_t blocks = (total + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 4096 ? 4096 : blocks);
  hipLaunchKernelGGL(k_pack_dgrad_kc, dim3((unsigned)blocks), dim3(256), 0, st, w, out, Co, C, R,
                     S, sh, sw, nclass, pc, kmax);
}

static ConvGeom to_device(const ConvGeomHost& h) {
  ConvGeom c{};
  c.Hin = h.Hin; c.Win = h.Win; c.C = h.C;
  c.sh = h.sh; c.sw = h.sw; c.dh = h.dh; c.dw = h.dw;
  c.Hout = h.Hout; c.Wout = h.Wout; c.osy = h.osy; c.osx = h.osx;
  c.nclass = h.nclass;
  for (int i = 0; i < h.nclass; ++i) {
    ConvClass& k = c.cls[i];
    k.TR = h.TR[i]; k.TS = h.TS[i]; k.oh = h.oh[i]; k.ow = h.ow[i];
    k.Hg = h.Hg[i]; k.Wg = h.Wg[i]; k.py = h.py[i]; k.px = h.px[i];
    k.M = h.M[i]; k.K = h.K[i]; k.b_off = h.b_off[i];
  }
  return c;
}

#define LW_LAUNCH(AKC, BKC, EPI, PRO, CVM) \
  hipLaunchKernelGGL((k_gemm<BM, BN, BK, AKC, BKC, EPI, PRO, CVM>), grid, dim3(GT), 0, st, k)

template <int BM, int BN, int BK, int CVM>
static void conv_tile(const GemmArgs& g, const GemmK& k, int epi, dim3 grid, hipStream_t st) {
  const bool pro = g.pro_scale != nullptr;
  if constexpr (CVM == CV_A) {
    if (!g.b_kcontig) {                                   // data gradient: Wt is [K][C]
      if (epi == EPI_BSTATS) LW_LAUNCH(true, false, EPI_BSTATS, PRO_NONE, CV_A);
      else LW_LAUNCH(true, false, EPI_STORE, PRO_NONE, CV_A);
    } else if (epi == EPI_STATS) {
      if (pro) LW_LAUNCH(true, true, EPI_STATS, PRO_A, CV_A);
      else LW_LAUNCH(true, true, EPI_STATS, PRO_NONE, CV_A);
    } else {
      if (pro) LW_LAUNCH(true, true, EPI_STORE, PRO_A, CV_A);
      else LW_LAUNCH(true, true, EPI_STORE, PRO_NONE, CV_A);
    }
  } else if constexpr (CVM == CV_A4) {
    if (epi == EPI_STATS) LW_LAUNCH(true, true, EPI_STATS, PRO_NONE, CV_A4);
    else LW_LAUNCH(true, true, EPI_STORE, PRO_NONE, CV_A4);
  } else if constexpr (CVM == CV_B) {            // (no prologue: the caller materialises)
    if (epi == EPI_PARTIAL) LW_LAUNCH(false, false, EPI_PARTIAL, PRO_NONE, CV_B);
    else LW_LAUNCH(false, false, EPI_STORE, PRO_NONE, CV_B);
  } else {
    if (epi == EPI_PARTIAL) LW_LAUNCH(false, false, EPI_PARTIAL, PRO_NONE, CV_B4);
    else LW_LAUNCH(false, false, EPI_STORE, PRO_NONE, CV_B4);
  }
}
#undef LW_LAUNCH

// Tile families: the row-gather passes (forward / dgrad: M = pixels, large) take the square and
// skinny-N tiles; the weight-gradient pass (M = Co, N = taps·C) the square and skinny-M ones.
void conv_big(const GemmArgs& g, const GemmK& k, hipStream_t st);     // gemm_big.hip

bool conv_tile_ok(int mode, int tile) {
  if (mode == CV_A && (tile == GEMM_B256 || tile == GEMM_B256x128)) return true;
  if (mode == CV_A || mode == CV_A4)
    return tile == GEMM_T128x128x32 || tile == GEMM_T128x128x64 || tile == GEMM_T256x64x32 ||
           tile == GEMM_T256x64x64 || tile == GEMM_T64x64x64;
  return tile == GEMM_T128x128x32 || tile == GEMM_T128x128x64 || tile == GEMM_T64x256x32 ||
         tile == GEMM_T64x64x64;
}

template <int CVM>
static void conv_dispatch(const GemmArgs& g, const GemmK& k, int epi, dim3 grid, hipStream_t st) {
  if constexpr (CVM == CV_A || CVM == CV_A4) {
    switch (g.tile) {
      case GEMM_T128x128x64: conv_tile<128, 128, 64, CVM>(g, k, epi, grid, st); break;
      case GEMM_T256x64x32: conv_tile<256, 64, 32, CVM>(g, k, epi, grid, st); break;
      case GEMM_T256x64x64: conv_tile<256, 64, 64, CVM>(g, k, epi, grid, st); break;
      case GEMM_T64x64x64: conv_tile<64, 64, 64, CVM>(g, k, epi, grid, st); break;
      default: conv_tile<128, 128, 32, CVM>(g, k, epi, grid, st); break;
    }
  } else {
    switch (g.tile) {
      case GEMM_T128x128x64: conv_tile<128, 128, 64, CVM>(g, k, epi, grid, st); break;
      case GEMM_T64x256x32: conv_tile<64, 256, 32, CVM>(g, k, epi, grid, st); break;
      case GEMM_T64x64x64: conv_tile<64, 64, 64, CVM>(g, k, epi, grid, st); break;
      default: conv_tile<128, 128, 32, CVM>(g, k, epi, grid, st); break;
    }
  }
}

int conv_splits_used(const GemmArgs& g) {
  int bm, bn, bk;
  gemm_tile_shape(g.tile, bm, bn, bk);
  const int kps = gemm_k_per_split(g.K, g.splits, bk);
  return (g.K + kps - 1) / kps;
}

void conv_gemm(const GemmArgs& g, const ConvGeomHost& cvh, int mode, hipStream_t st) {
  int bm, bn, bk;
  gemm_tile_shape(g.tile, bm, bn, bk);
  const int kps = gemm_k_per_split(g.K, g.splits, bk);
  const int zs = (g.K + kps - 1) / kps;
  const int tiles = ((g.M + bm - 1) / bm) * ((g.N + bn - 1) / bn);
  const int epi = zs > 1 ? EPI_PARTIAL
                          : (g.stats ? (g.bst_x ? EPI_BSTATS : EPI_STATS) : EPI_STORE);
  GemmK k{g.A, g.B, g.C, g.partial, g.stats, zs > 1 ? nullptr : g.bias, g.pro_scale, g.pro_shift,
          g.addend, nullptr, g.lda, g.ldb, g.ldc, g.M, g.N, g.K, kps, zs > 1 ? 0 : (g.relu ? 1 : 0),
          g.out_bf16 ? 1 : 0, g.accumulate ? 1 : 0};
  k.cv = to_device(cvh);
  k.a_bytes = g.a_bytes;
  k.b_bytes = g.b_bytes;
  k.bst_x = g.bst_x;
  k.bst_mean = g.bst_mean;
  k.bst_scale = g.bst_scale;
  k.bst_shift = g.bst_shift;
  k.bst_bits = g.bst_bits;
  if (g.tile == GEMM_B256 || g.tile == GEMM_B256x128) {
    conv_big(g, k, st);              // (bindings.cpp checked conv_big_ok)
    return;
  }
  const dim3 grid(tiles, zs, cvh.nclass);
  switch (mode) {
    case CV_A: conv_dispatch<CV_A>(g, k, epi, grid, st); break;
    case CV_A4: conv_dispatch<CV_A4>(g, k, epi, grid, st); break;
    case CV_B: conv_dispatch<CV_B>(g, k, epi, grid, st); break;
    default: conv_dispatch<CV_B4>(g, k, epi, grid, st); break;
  }
  if (zs > 1) splitk_reduce(g, zs, st);
}

}  // namespace lw
