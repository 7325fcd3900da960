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
bool conv_tile_ok(int mode, int tile) {
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
