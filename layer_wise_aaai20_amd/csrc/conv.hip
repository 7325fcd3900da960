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

// Several data-gradient weight packs in one launch (ops/conv.py kc_pack: the packed weights of a
// step — 1x1 transposes, strided / 3x3 class slabs, flipped 3x3 windows, [K][C] slabs — made once
// per step at the first request instead of one launch each). Per job the body of k_pack_dgrad_kc,
// or of k_pack_dgrad_nkc for kmax == 0.
struct KcJob {
  const uint16_t* w;
  uint16_t* out;
  int Co, C, R, S, sh, sw, nclass, kmax;
  PackClasses pc;
  int64_t blk_lo;
};
constexpr int kMaxKcJobs = 24;
struct KcJobs {
  KcJob j[kMaxKcJobs];
  int n;
};

__global__ __launch_bounds__(256) void k_pack_kc_multi(const KcJobs jobs) {
  int ji = 0;
  for (int q = 1; q < jobs.n; ++q)
    if ((int64_t)blockIdx.x >= jobs.j[q].blk_lo) ji = q;
  const KcJob& J = jobs.j[ji];
  int64_t t = ((int64_t)blockIdx.x - J.blk_lo) * 256 + threadIdx.x;
  if (J.kmax == 0) {                 // the [K][C] form: k_pack_dgrad_nkc's body, 16-byte chunks
    const int C8 = J.C / 8;
    int64_t base = 0;
    for (int i = 0; i < J.nclass; ++i) {
      const int r0 = i == 0 ? J.pc.r0[0] : i == 1 ? J.pc.r0[1] : i == 2 ? J.pc.r0[2] : J.pc.r0[3];
      const int s0 = i == 0 ? J.pc.s0[0] : i == 1 ? J.pc.s0[1] : i == 2 ? J.pc.s0[2] : J.pc.s0[3];
      const int TR = i == 0 ? J.pc.TR[0] : i == 1 ? J.pc.TR[1] : i == 2 ? J.pc.TR[2] : J.pc.TR[3];
      const int TS = i == 0 ? J.pc.TS[0] : i == 1 ? J.pc.TS[1] : i == 2 ? J.pc.TS[2] : J.pc.TS[3];
      const int64_t n = (int64_t)TR * TS * J.Co * C8;
      if (t < n) {
        const int cg = (int)(t % C8);
        const int64_t row = t / C8;                      // (jr, js, co)
        const int o = (int)(row % J.Co);
        const int tap = (int)(row / J.Co);
        const int jr = tap / TS, js = tap - jr * TS;
        const int r = r0 + J.sh * jr, sx = s0 + J.sw * js;
        const uint4 v = *reinterpret_cast<const uint4*>(
            J.w + (((int64_t)o * J.R + r) * J.S + sx) * J.C + cg * 8);
        *reinterpret_cast<uint4*>(J.out + base + row * J.C + cg * 8) = v;
        return;
      }
      t -= n;
      base += (int64_t)TR * TS * J.Co * J.C;
    }
    return;
  }
  const int64_t per_row = J.kmax / 8, per_class = (int64_t)J.C * per_row;
  if (t >= J.nclass * per_class) return;
  const int i = (int)(t / per_class);
  const int64_t rem = t - i * per_class;
  const int c = (int)(rem / per_row);
  const int k0 = (int)(rem - (int64_t)c * per_row) * 8;
  const int r0 = i == 0 ? J.pc.r0[0] : i == 1 ? J.pc.r0[1] : i == 2 ? J.pc.r0[2] : J.pc.r0[3];
  const int s0 = i == 0 ? J.pc.s0[0] : i == 1 ? J.pc.s0[1] : i == 2 ? J.pc.s0[2] : J.pc.s0[3];
  const int TR = i == 0 ? J.pc.TR[0] : i == 1 ? J.pc.TR[1] : i == 2 ? J.pc.TR[2] : J.pc.TR[3];
  const int TS = i == 0 ? J.pc.TS[0] : i == 1 ? J.pc.TS[1] : i == 2 ? J.pc.TS[2] : J.pc.TS[3];
  const int Kc = TR * TS * J.Co;
  uint16_t v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int k = k0 + q;
    uint16_t x = 0;
    if (k < Kc) {
      const int tap = k / J.Co, o = k - tap * J.Co;
      const int jr = tap / TS, js = tap - jr * TS;
      const int r = r0 + J.sh * jr, sx = s0 + J.sw * js;
      x = J.w[(((int64_t)o * J.R + r) * J.S + sx) * J.C + c];
    }
    v[q] = x;
  }
  *reinterpret_cast<uint4*>(J.out + (int64_t)i * J.C * J.kmax + (int64_t)c * J.kmax + k0) =
      make_uint4((uint32_t)v[0] | ((uint32_t)v[1] << 16), (uint32_t)v[2] | ((uint32_t)v[3] << 16),
                 (uint32_t)v[4] | ((uint32_t)v[5] << 16), (uint32_t)v[6] | ((uint32_t)v[7] << 16));
}

// prm: per job [Co, C, R, S, sh, sw, nclass, kmax, r0 x4, s0 x4, TR x4, TS x4] (24 ints)
void pack_kc_multi(const uint16_t* const* w, uint16_t* const* out, const int* prm, int n,
                   hipStream_t st) {
  for (int b = 0; b < n; b += kMaxKcJobs) {
    KcJobs jobs{};
    jobs.n = n - b < kMaxKcJobs ? n - b : kMaxKcJobs;
    int64_t blocks = 0;
    for (int q = 0; q < jobs.n; ++q) {
      const int* p = prm + 24 * (b + q);
      KcJob J{};
      J.w = w[b + q];
      J.out = out[b + q];
      J.Co = p[0]; J.C = p[1]; J.R = p[2]; J.S = p[3]; J.sh = p[4]; J.sw = p[5];
      J.nclass = p[6]; J.kmax = p[7];
      for (int i = 0; i < 4; ++i) {
        J.pc.r0[i] = p[8 + i]; J.pc.s0[i] = p[12 + i]; J.pc.TR[i] = p[16 + i]; J.pc.TS[i] = p[20 + i];
      }
      J.blk_lo = blocks;
      int64_t chunks = (int64_t)J.nclass * J.C * (J.kmax / 8);
      if (J.kmax == 0) {
        chunks = 0;
        for (int i = 0; i < J.nclass; ++i)
          chunks += (int64_t)J.pc.TR[i] * J.pc.TS[i] * J.Co * (J.C / 8);
      }
      blocks += (chunks + 255) / 256;
      jobs.j[q] = J;
    }
    hipLaunchKernelGGL(k_pack_kc_multi, dim3((unsigned)blocks), dim3(256), 0, st, jobs);
  }
}

// The [K][C] form (the data-gradient GEMM's B operand read with the transposing LDS loads): class
// i's slab Wt_i[jr][js][co][ci] = w[co][r0 + sh*jr][s0 + sw*js][ci], slabs back to back. Each
// thread moves 8 consecutive ci (one 16-byte load and store; C % 8 == 0). Replaces a permute +
// per-class slice copies + concatenation (up to 5 ATen kernels per stride-2 layer).
__global__ __launch_bounds__(256) void k_pack_dgrad_nkc(const uint16_t* __restrict__ w,
                                                        uint16_t* __restrict__ out, int Co, int C,
                                                        int R, int S, int sh, int sw, int nclass,
                                                        PackClasses pc) {
  const int C8 = C / 8;
  int64_t base = 0;
  for (int i = 0; i < nclass; ++i) {
    const int r0 = pc.r0[i], s0 = pc.s0[i], TR = pc.TR[i], TS = pc.TS[i];
    const int64_t n = (int64_t)TR * TS * Co * C8;      // 16-byte chunks of this class
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n;
         t += (int64_t)gridDim.x * 256) {
      const int cg = (int)(t % C8);
      const int64_t row = t / C8;                        // (jr, js, co)
      const int o = (int)(row % Co);
      const int tap = (int)(row / Co);
      const int jr = tap / TS, js = tap - jr * TS;
      const int r = r0 + sh * jr, sx = s0 + sw * js;
      const uint4 v = *reinterpret_cast<const uint4*>(w + (((int64_t)o * R + r) * S + sx) * C +
                                                      cg * 8);
      *reinterpret_cast<uint4*>(out + base + row * C + cg * 8) = v;
    }
    base += (int64_t)TR * TS * Co * C;
  }
}

void pack_dgrad_nkc(const uint16_t* w, uint16_t* out, int Co, int C, int R, int S, int sh, int sw,
                    int nclass, const int* r0, const int* s0, const int* TR, const int* TS,
                    hipStream_t st) {
  PackClasses pc{};
  int64_t most = 1;
  for (int i = 0; i < nclass; ++i) {
    pc.r0[i] = r0[i]; pc.s0[i] = s0[i]; pc.TR[i] = TR[i]; pc.TS[i] = TS[i];
    const int64_t n = (int64_t)TR[i] * TS[i] * Co * (C / 8);
    most = n > most ? n : most;
  }
  int64_t blocks = (most + 255) / 256;
  blocks = blocks > 4096 ? 4096 : blocks;
  hipLaunchKernelGGL(k_pack_dgrad_nkc, dim3((unsigned)blocks), dim3(256), 0, st, w, out, Co, C, R,
                     S, sh, sw, nclass, pc);
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
  hipLaunchKernelGGL((k_gemm<BM, BN, BK, AKC, BKC, EPI, PRO, CVM, MF>), grid, dim3(GT), 0, st, k)

template <int BM, int BN, int BK, int CVM, int MF>
static void conv_tile(const GemmArgs& g, const GemmK& k, int epi, dim3 grid, hipStream_t st) {
  const bool pro = g.pro_scale != nullptr;
  if constexpr (CVM == CV_A) {
    if (!g.b_kcontig) {                                   // data gradient: Wt is [K][C]
      LW_LAUNCH(true, false, EPI_STORE, PRO_NONE, CV_A);
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
void conv_big(const GemmArgs& g, const GemmK& k, int zs, hipStream_t st);   // gemm_big.hip

bool conv_tile_ok(int mode, int tile) {
  if ((mode == CV_A || mode == CV_B) && (tile == GEMM_B256 || tile == GEMM_B256x128)) return true;
  tile = gemm_base_tile(tile);         // the MF = 32 twins are built for the same tiles
  if (mode == CV_A || mode == CV_A4)
    return tile == GEMM_T128x128x32 || tile == GEMM_T128x128x64 || tile == GEMM_T256x64x32 ||
           tile == GEMM_T256x64x64 || tile == GEMM_T64x64x64;
  return tile == GEMM_T128x128x32 || tile == GEMM_T128x128x64 || tile == GEMM_T64x256x32 ||
         tile == GEMM_T64x64x64;
}

template <int CVM, int MF>
static void conv_dispatch_mf(const GemmArgs& g, const GemmK& k, int epi, dim3 grid,
                             hipStream_t st) {
  if constexpr (CVM == CV_A || CVM == CV_A4) {
    switch (gemm_base_tile(g.tile)) {
      case GEMM_T128x128x64: conv_tile<128, 128, 64, CVM, MF>(g, k, epi, grid, st); break;
      case GEMM_T256x64x32: conv_tile<256, 64, 32, CVM, MF>(g, k, epi, grid, st); break;
      case GEMM_T256x64x64: conv_tile<256, 64, 64, CVM, MF>(g, k, epi, grid, st); break;
      case GEMM_T64x64x64: conv_tile<64, 64, 64, CVM, MF>(g, k, epi, grid, st); break;
      default: conv_tile<128, 128, 32, CVM, MF>(g, k, epi, grid, st); break;
    }
  } else {
    switch (gemm_base_tile(g.tile)) {
      case GEMM_T128x128x64: conv_tile<128, 128, 64, CVM, MF>(g, k, epi, grid, st); break;
      case GEMM_T64x256x32: conv_tile<64, 256, 32, CVM, MF>(g, k, epi, grid, st); break;
      case GEMM_T64x64x64: conv_tile<64, 64, 64, CVM, MF>(g, k, epi, grid, st); break;
      default: conv_tile<128, 128, 32, CVM, MF>(g, k, epi, grid, st); break;
    }
  }
}

template <int CVM>
static void conv_dispatch(const GemmArgs& g, const GemmK& k, int epi, dim3 grid, hipStream_t st) {
  if (gemm_is_mf32(g.tile)) conv_dispatch_mf<CVM, 32>(g, k, epi, grid, st);
  else conv_dispatch_mf<CVM, 16>(g, k, epi, grid, st);
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
    conv_big(g, k, zs, st);          // (bindings.cpp checked conv_big_ok)
    if (zs > 1) splitk_reduce(g, zs, st);
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

namespace lw {

// ---------------------------------------------------------------------------------------------
// The ResNet stem convolution (7x7, stride 2, pad 3, a 3-channel image padded to 4, 64 output
// channels) as a direct convolution from an LDS patch. The implicit GEMM above gathers every
// im2col chunk of this K = 7x8x4 = 224 problem from L2 with two 8-byte loads (its N = 64 output
// channels reuse each chunk only 4 times), which left it at ~130 TFLOP/s. Here a workgroup owns
// SY output rows of one image: it stages the (2*SY + 5) x (2*Wo + 6) x 4 input patch (zero
// padding included) and the packed weight [64][224] in LDS once, and every MFMA operand is one
// ds_read_b128: for output pixel (y, x), filter row r and tap pair (2g, 2g + 1) the 8 values
// (2 taps x 4 channels) are adjacent in the patch row 2y + r at columns 2x + 2g, 2x + 2g + 1.
// The k order (r, tap, channel) and the 32-wide MFMA steps are those of the GEMM path's packed
// weight (pack_fwd_weight), so the outputs are bit-identical to it. Epilogue: bf16 NHWC store and
// one column-statistics row (Σv, Σv² of the stored values) per workgroup.
// A workgroup walks `tpw` consecutive row tiles: the packed weight is staged once, and the next
// tile's patch is loaded into registers (all its loads in flight at once) while the MFMAs of the
// current tile run, so the staging latency is paid once per workgroup instead of once per tile
// (the one-tile-per-workgroup form waited on ~11 serial global round trips per tile).
constexpr int STEM_SY = 4;                 // output rows per tile
constexpr int STEM_CO = 64;
constexpr int STEM_K = 224;                // 7 rows x 8 taps (7 + 1 zero) x 4 channels
constexpr int STEM_WLD = STEM_K + 8;       // padded LDS weight row (bank spread)
constexpr int STEM_WAVES = 7;              // 448 threads: 28 pixel blocks of 16 = 4 per wave
constexpr int STEM_T = STEM_WAVES * 64;
constexpr int STEM_WOMAX = 112;            // widest output row (224 px images)
constexpr int STEM_PW = 2 * STEM_WOMAX + 6;  // patch row pitch (pixels): a compile-time stride, so
                                           // every patch read is one base + immediate offset
constexpr int STEM_PR = 2 * STEM_SY + 5;   // patch rows
constexpr int STEM_PMAX = (STEM_PR * STEM_PW + STEM_T - 1) / STEM_T;   // patch pixels per thread

// OCC: waves per SIMD the register allocation targets (4 = two workgroups per CU at 128 VGPRs,
// a few spills; 3 = no spills, one workgroup per CU). PF: the next tile's patch loads are issued
// before this tile's MFMAs (held in registers across them) instead of at the top of each tile.
template <int OCC, bool PF>
__global__ __launch_bounds__(STEM_T) __attribute__((amdgpu_waves_per_eu(OCC))) void k_stem_conv7(const uint16_t* __restrict__ x,
                                                    const uint16_t* __restrict__ w,
                                                    uint16_t* __restrict__ y,
                                                    float* __restrict__ stats, int H, int W,
                                                    int Ho, int Wo, int tiles, int tpw) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int PW = STEM_PW, PR = STEM_PR;       // columns past 2 * Wo + 6 are never read
  uint16_t* patch = reinterpret_cast<uint16_t*>(smem);               // [PR][PW][4]
  uint16_t* ws = patch + PR * PW * 4;                                 // [64][STEM_WLD]
  float* red = reinterpret_cast<float*>(ws + STEM_CO * STEM_WLD);     // [waves][2][64]
  const int tiles_y = Ho / STEM_SY;
  const int t0 = blockIdx.x * tpw, t1 = min(t0 + tpw, tiles);
  // this thread's patch pixels e = tid + i * STEM_T, walked as (row, column) with a carry (kept
  // out of registers across the tile loop)
  const int prow0 = threadIdx.x / PW, pcol0 = threadIdx.x - prow0 * PW;
  const int dq = STEM_T / PW, dr = STEM_T - dq * PW;
  uint2 pv[STEM_PMAX];
  auto load_patch = [&](int t) {                   // 8-byte pixels; outside the image: zeros
    const int img = t / tiles_y, y0 = (t - img * tiles_y) * STEM_SY;
    const uint16_t* xi = x + (int64_t)img * H * W * 4;
    int pr = prow0, pc = pcol0;
#pragma unroll
    for (int i = 0; i < STEM_PMAX; ++i) {
      const int hi = 2 * y0 - 3 + pr, wi = pc - 3;
      pv[i] = make_uint2(0u, 0u);
      if (pr < PR && (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W)
        pv[i] = *reinterpret_cast<const uint2*>(xi + ((int64_t)hi * W + wi) * 4);
      pc += dr; pr += dq;
      if (pc >= PW) { pc -= PW; ++pr; }
    }
  };
  {
    constexpr int WPT = STEM_CO * (STEM_K / 8) / STEM_T;      // 4 uint4 per thread
    static_assert(STEM_CO * (STEM_K / 8) == WPT * STEM_T, "weight staging");
    uint4 wv[WPT];
#pragma unroll
    for (int i = 0; i < WPT; ++i) {
      const int e = threadIdx.x + i * STEM_T;
      const int co = e / (STEM_K / 8), kc = e - co * (STEM_K / 8);
      wv[i] = *reinterpret_cast<const uint4*>(w + co * STEM_K + kc * 8);
    }
#pragma unroll
    for (int i = 0; i < WPT; ++i) {
      const int e = threadIdx.x + i * STEM_T;
      const int co = e / (STEM_K / 8), kc = e - co * (STEM_K / 8);
      *reinterpret_cast<uint4*>(ws + co * STEM_WLD + kc * 8) = wv[i];
    }
  }
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, lr = l & 15;
  const int npix = STEM_SY * Wo;                   // STEM_WAVES * 16 * RB (host)
  const int RB = npix / (STEM_WAVES * 16);         // 16-row blocks per wave
  constexpr int MAXRB = 4;
  // this lane's pixel of row block i: wave wv takes blocks wv, wv + STEM_WAVES, ...
  int poff[MAXRB];
#pragma unroll
  for (int i = 0; i < MAXRB; ++i) {
    const int p = (wv + STEM_WAVES * i) * 16 + lr;
    const int yy = p / Wo, xx = p - yy * Wo;
    poff[i] = ((2 * yy) * PW + 2 * xx + 2 * g) * 4;   // element offset at filter row 0
  }
  // column statistics: each wave folds its tile sums into its own [2][64] LDS row (no races)
  for (int c = l; c < 2 * STEM_CO; c += 64) red[wv * 2 * STEM_CO + c] = 0.f;
  if (PF && t0 < t1) load_patch(t0);
  for (int t = t0; t < t1; ++t) {
    if (!PF) load_patch(t);                        // all loads in flight at once
    __syncthreads();                               // the previous tile's patch reads are done
#pragma unroll
    for (int i = 0; i < STEM_PMAX; ++i) {
      const int e = threadIdx.x + i * STEM_T;
      if (e < PR * PW) *reinterpret_cast<uint2*>(patch + e * 4) = pv[i];
    }
    __syncthreads();
    if (PF && t + 1 < t1) load_patch(t + 1);       // in flight under this tile's MFMAs
    f32x4 acc[MAXRB][4];
#pragma unroll
    for (int i = 0; i < MAXRB; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < 7; ++r) {
      h16x8 fb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        fb[j] = *reinterpret_cast<const h16x8*>(ws + (j * 16 + lr) * STEM_WLD + r * 32 + g * 8);
#pragma unroll
      for (int i = 0; i < MAXRB; ++i) {
        if (i < RB) {
          const h16x8 fa = *reinterpret_cast<const h16x8*>(patch + poff[i] + r * PW * 4);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = mfma16(fb[j], fa, acc[i][j]);
        }
      }
    }
    // ---- epilogue: lane holds C[pixel (l & 15)][channel 4 * (l >> 4) + q] of each 16x16 block
    const int img = t / tiles_y, y0 = (t - img * tiles_y) * STEM_SY;
    const int64_t out_base = ((int64_t)img * Ho + y0) * Wo;       // first pixel of the tile
    // channel block j at a time (its 4 statistics pairs only live across the row blocks)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < MAXRB; ++i) {
        if (i >= RB) continue;
        const int p = (wv + STEM_WAVES * i) * 16 + lr;
        uint16_t h[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          h[q] = f2h(acc[i][j][q]);
          const float v = h2f(h[q]);
          s1[q] += v;
          s2[q] += v * v;
        }
        *reinterpret_cast<uint2*>(y + (out_base + p) * STEM_CO + j * 16 + 4 * g) =
            make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16));
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        s1[q] = sum16(s1[q]);
        s2[q] = sum16(s2[q]);
      }
      if (lr == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          red[(wv * 2 + 0) * STEM_CO + j * 16 + 4 * g + q] += s1[q];
          red[(wv * 2 + 1) * STEM_CO + j * 16 + 4 * g + q] += s2[q];
        }
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 * STEM_CO) {
    const int sidx = threadIdx.x / STEM_CO, c = threadIdx.x - sidx * STEM_CO;
    float tsum = 0.f;
#pragma unroll
    for (int q = 0; q < STEM_WAVES; ++q) tsum += red[(q * 2 + sidx) * STEM_CO + c];   // fixed order
    stats[((int64_t)blockIdx.x * 2 + sidx) * STEM_CO + c] = tsum;
  }
}

int stem_conv7_smem(int) {
  return STEM_PR * STEM_PW * 4 * 2 + STEM_CO * STEM_WLD * 2 + STEM_WAVES * 2 * STEM_CO * 4;
}

bool stem_conv7_ok(int C, int Co, int R, int S, int sh, int sw, int ph, int pw, int H, int W,
                   int Ho, int Wo) {
  return C == 4 && Co == STEM_CO && R == 7 && S == 7 && sh == 2 && sw == 2 && ph == 3 && pw == 3 &&
         Ho == (H + 6 - 7) / 2 + 1 && Wo == (W + 6 - 7) / 2 + 1 && Ho % STEM_SY == 0 &&
         (STEM_SY * Wo) % (STEM_WAVES * 16) == 0 && STEM_SY * Wo / (STEM_WAVES * 16) <= 4 &&
         Wo <= STEM_WOMAX && stem_conv7_smem(Wo) <= 64 * 1024;
}

// tiles per workgroup: enough workgroups for two resident per CU (the LDS footprint allows two)
static int stem_tpw(int tiles) {
  const int slots = 2 * cu_count();
  return std::max(1, (tiles + slots - 1) / slots);
}

int stem_conv7_blocks(int N, int Ho) {
  const int tiles = N * (Ho / STEM_SY);
  const int tpw = stem_tpw(tiles);
  return (tiles + tpw - 1) / tpw;
}

void stem_conv7(const uint16_t* x, const uint16_t* w, uint16_t* y, float* stats, int N, int H,
                int W, int Ho, int Wo, hipStream_t st) {
  const int tiles = N * (Ho / STEM_SY);
  const int tpw = stem_tpw(tiles);
  const int blocks = (tiles + tpw - 1) / tpw;
  // (the next-tile patch prefetch and 3 waves/SIMD variants were faster in isolation, 213 vs
  // 251 us, but not in the step: profiles/r3s2/stem_ab.txt; round 6 removed them)
  hipLaunchKernelGGL((k_stem_conv7<4, false>), dim3(blocks), dim3(STEM_T), stem_conv7_smem(Wo), st,
                     x, w, y, stats, H, W, Ho, Wo, tiles, tpw);
}

}  // namespace lw
