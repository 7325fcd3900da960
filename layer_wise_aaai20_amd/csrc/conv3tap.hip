// Tap-reuse 3x3 / stride-1 / pad-1 convolution for gfx950 (ResNet bottleneck conv2, every conv of
// the CIFAR networks): forward, and — with the flipped, transposed weight — the data gradient.
//
// Why: the implicit GEMM (conv.hip) gathers each input chunk from L2 once per filter tap, i.e. 9
// times. Its 128x128 tiles then move 32 KB through L2 -> LDS per 2.1 MFLOP, which is the per-CU
// gather rate at 2 workgroups per CU (~70 GB/s/CU, MI355X_MICROARCH.md "gather into LDS"): the
// 3x3 convolutions ran at 390-610 TFLOP/s whatever the MFMA schedule (profiles/r3s2
// op_roofline_splitxcd.txt). Here the input patch of a tile is staged once per 32-channel chunk and
// read by all 9 taps, so the operand traffic per FLOP drops ~4-8x and the MFMAs set the pace.
//
// Tile: T3_M = 224 output pixels = whole rows (every image width of the supported models divides
// 224: 56, 28, 14, 7, 32, 16, 8, 4) x BN output channels (64 or 128). Rows are global rows of the
// [N*H] row space, so a tile may span images: a tap row that falls outside the pixel's own image
// reads as zero (per-lane mask on the A fragment), the halo columns are zero in the patch.
// K order: (chunk c of 32 channels) outer, tap (r, s) inner; each K-step is one 16x16x32 MFMA
// k-step, so the arithmetic is the GEMM path's up to the order of the fp32 sums.
//
// LDS (per workgroup, 2 workgroups per CU): two 24 KB patch buffers [pixel][4 x 16 B] (chunk c and
// c + 1) and a ring of 3 weight slices [BN][4 x 16 B] (K-steps s, s + 1, s + 2), all filled by
// LDS-DMA (buffer_load ... lds) with the XOR swizzle applied on the SOURCE side:
//   patch: the 16-byte slot of 8-channel group g of patch pixel p is g ^ ((p >> 2) & 3), so the
//          16 consecutive pixels an MFMA fragment read touches hit 16 distinct bank groups;
//   weight: slot of group g of row n is g ^ ((n >> 2) & 3) (same argument over 16 rows).
// Schedule per K-step s = (c, t): DMA weight slice s + 2; at t == 4 DMA the next chunk's patch;
// 7 A + 2 B fragment reads (per wave: 7 pixel blocks x 2 channel blocks), 14 MFMAs; counted
// s_waitcnt vmcnt for the slice (and patch) the next step reads; one barrier.
// Epilogue: the tile is staged as bf16 in LDS, stored in 16-byte chunks, and (forward) the column
// statistics Σv, Σv² of the stored values are written as one row per 224-pixel tile ([tiles][2][Co],
// the layout of the GEMM epilogue's statistics rows).
#include "gemm_core.h"

namespace lw {

constexpr int T3_M = 224;                 // output pixels per tile
constexpr int T3_PATCH = 24 * 1024;       // bytes per patch buffer (one 32-channel chunk)
constexpr int T3_NWS = 3;                 // weight slices in the ring

template <int N>
__device__ __forceinline__ void t3_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// BN output channels per workgroup (BN / 16 waves: 2 pixel halves x BN / 32 channel groups)
template <int BN, bool STATS>
__global__ __launch_bounds__(BN * 4) __attribute__((amdgpu_waves_per_eu(BN == 128 ? 4 : 2)))
void k_conv3_tap(const uint16_t* __restrict__ x,
                                                         const uint16_t* __restrict__ w,
                                                         uint16_t* __restrict__ y,
                                                         float* __restrict__ stats, int NH, int H,
                                                         int W, int C, int Co, uint32_t x_bytes,
                                                         uint32_t w_bytes) {
  constexpr int NT = BN * 4;                       // threads
  constexpr int NWAVE = BN / 16;
  constexpr int NPJ = T3_PATCH / (NWAVE * 1024);   // patch DMA instructions per thread
  constexpr int WSL = BN * 64;                     // bytes per weight slice (BN rows x 32 k)
  constexpr int LDS = 2 * T3_PATCH + T3_NWS * WSL;
  constexpr int LDH = BN + 8;                      // bf16 staging row (epilogue)
  static_assert(T3_M * LDH * 2 <= LDS, "epilogue staging fits the ring");
  static_assert(NT * 16 * 4 <= LDS, "statistics fold fits");
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS];

  const int R = T3_M / W, PW = W + 2, npix = (R + 2) * PW;
  const int tiles_n = Co / BN;
  const int total = gridDim.x;
  const int pid = xcd_remap((int)blockIdx.x, total);   // the n-tiles of one m-tile share an XCD
  const int tm = pid / tiles_n, tn = pid - tm * tiles_n;
  const int g0 = tm * R;                          // first output row (global row space)
  const int n0 = tn * BN;
  const int NC = C / 32, S = 9 * NC;
  const int64_t K = 9 * (int64_t)C;
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int wm = wave & 1, wn = wave >> 1;        // pixel half (7 blocks), 32-channel group
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(x, x_bytes), rw = make_rsrc(w, w_bytes);

  // ---- per-thread DMA sources. Patch: instruction j lands 16-byte chunk q = (j*NWAVE + wave)*64
  // + lane: pixel p = q >> 2, slot q & 3, fetching channel group (q & 3) ^ ((p >> 2) & 3)
  int prel[NPJ], prow[NPJ];                        // byte offset rel. to (row g0-1, chunk 0); row
  uint32_t pok = 0;                                // pixel inside the patch and its column in W
#pragma unroll
  for (int j = 0; j < NPJ; ++j) {
    const int q = (j * NWAVE + wave) * 64 + l;
    const int p = q >> 2, slot = q & 3, gs = slot ^ ((p >> 2) & 3);
    const int pr = p / PW, pc = p - pr * PW;
    prow[j] = pr;
    prel[j] = ((pr * W + pc - 1) * C + gs * 8) * 2;
    pok |= (p < npix && pc >= 1 && pc <= W ? 1u : 0u) << j;
  }
  // (g0 - 1) * row bytes, modulo 2^32: row -1 is never fetched, and every fetched offset is
  // < 2^31 (checked on the host), so 32-bit wrap-around arithmetic gives the exact offset
  const uint32_t tile_base = (uint32_t)(g0 - 1) * (uint32_t)(W * C * 2);
  auto issue_patch = [&](int c, int buf) {
    uint8_t* dst = lds + buf * T3_PATCH;
#pragma unroll
    for (int j = 0; j < NPJ; ++j) {
      const int G = g0 - 1 + prow[j];
      const bool ok = ((pok >> j) & 1u) && G >= 0 && G < NH;
      const uint32_t off = ok ? tile_base + (uint32_t)prel[j] + (uint32_t)(c * 64) : OOB;
      glds16(rx, reinterpret_cast<uint16_t*>(dst + (j * NWAVE + wave) * 1024), off);
    }
  };
  // weight slice of K-step s = (c, t): rows n0 + wave*16 + (lane >> 2), k = t*C + c*32 + 8*g
  const int wrow = wave * 16 + (l >> 2);
  const int wgs = (l & 3) ^ ((wrow >> 2) & 3);
  const uint32_t wrel = (uint32_t)(((int64_t)(n0 + wrow) * K + wgs * 8) * 2);
  auto issue_w = [&](int s, int slot) {
    const int c = s / 9, t = s - c * 9;
    uint32_t wr = wrel;
    asm volatile("" : "+v"(wr));                   // (not hoisted per step: registers)
    const uint32_t off = wr + (uint32_t)((t * C + c * 32) * 2);
    glds16(rw, reinterpret_cast<uint16_t*>(lds + 2 * T3_PATCH + slot * WSL + wave * 1024), off);
  };

  // ---- per-lane fragment geometry: pixel blocks wm*7 + i, lane pixel (l & 15); k group g
  const int g = l >> 4;
  int ppix[7];                 // patch pixel of tap (0, 0)
  uint32_t rmask = 0;          // bit 2i: tap row 0 inside the image; bit 2i+1: tap row 2
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int m = (wm * 7 + i) * 16 + (l & 15);
    const int orow = m / W, ox = m - orow * W;
    ppix[i] = orow * PW + ox;
    const int yy = (g0 + orow) % H;
    rmask |= (yy >= 1 ? 1u : 0u) << (2 * i);
    rmask |= (yy + 1 < H ? 1u : 0u) << (2 * i + 1);
  }
  int wbyte[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = wn * 32 + j * 16 + (l & 15);
    wbyte[j] = (n * 4 + (g ^ ((n >> 2) & 3))) * 16;
  }

  f32x4 acc[7][2];
#pragma unroll
  for (int i = 0; i < 7; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const uint8_t* P, const uint8_t* Wt, int r, int s) {
    bf16x8 fb[2], fa[7];
#pragma unroll
    for (int j = 0; j < 2; ++j) fb[j] = *reinterpret_cast<const bf16x8*>(Wt + wbyte[j]);
    const int toff = r * PW + s;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      // opaque base: keeps the 63 (block, tap) addresses from being hoisted out of the K loop
      // into registers (they would spill)
      int pb = ppix[i];
      asm volatile("" : "+v"(pb));
      const int p = pb + toff;
      fa[i] = *reinterpret_cast<const bf16x8*>(P + (p * 4 + (g ^ ((p >> 2) & 3))) * 16);
      if (r != 1) {
        const bool ok = (rmask >> (2 * i + (r >> 1))) & 1u;
        if (!ok) fa[i] = bf16x8{};
      }
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 7; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // ---- prologue: patch of chunk 0, weight slices 0 and 1
  issue_patch(0, 0);
  issue_w(0, 0);
  if (S > 1) issue_w(1, 1);
  if (S > 1) t3_wait_barrier<1>();
  else t3_wait_barrier<0>();
  int slot = 0;
#pragma unroll 1
  for (int c = 0; c < NC; ++c) {
    const uint8_t* P = lds + (c & 1) * T3_PATCH;
    const bool next_chunk = c + 1 < NC;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int s = c * 9 + t;
      const bool w2 = s + 2 < S;
      if (w2) issue_w(s + 2, slot == 0 ? 2 : slot - 1);        // (s + 2) % 3
      if (t == 4 && next_chunk) issue_patch(c + 1, (c + 1) & 1);
      compute(P, lds + 2 * T3_PATCH + slot * WSL, t / 3, t % 3);
      // DMAs issued after slice s + 1 may stay in flight (loads retire in order)
      if ((t == 4 || t == 5) && next_chunk) {
        if (w2) t3_wait_barrier<NPJ + 1>();
        else t3_wait_barrier<NPJ>();
      } else {
        if (w2) t3_wait_barrier<1>();
        else t3_wait_barrier<0>();
      }
      slot = slot == 2 ? 0 : slot + 1;
    }
  }

  // ---- epilogue: bf16 tile staged in LDS, 16-byte stores, column statistics
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  uint16_t* Ch = reinterpret_cast<uint16_t*>(lds);
#pragma unroll
  for (int i = 0; i < 7; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int m = (wm * 7 + i) * 16 + (l & 15);
      const int n = wn * 32 + j * 16 + 4 * g;
      uint16_t h[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) h[r] = bf16_rne(acc[i][j][r]);
      *reinterpret_cast<uint2*>(Ch + m * LDH + n) =
          make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16));
    }
  __syncthreads();
  constexpr int CPR = BN / 8;                      // 16-byte chunks per row
  const int m_valid = min(T3_M, (NH - g0) * W);
  const int cg = threadIdx.x % CPR;                // this thread's 8 columns (fixed)
  float s1[8], s2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { s1[k] = 0.f; s2[k] = 0.f; }
  const int64_t m0 = (int64_t)g0 * W;
  for (int ch = threadIdx.x; ch < T3_M * CPR; ch += NT) {
    const int m = ch / CPR;
    if (m >= m_valid) break;                       // rows past the last are all at the end
    const uint4 v = *reinterpret_cast<const uint4*>(Ch + m * LDH + cg * 8);
    *reinterpret_cast<uint4*>(y + (m0 + m) * Co + n0 + cg * 8) = v;
    if constexpr (STATS) {
      const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float f = k & 1 ? __uint_as_float(u[k >> 1] & 0xffff0000u) : __uint_as_float(u[k >> 1] << 16);
        s1[k] += f;
        s2[k] += f * f;
      }
    }
  }
  if constexpr (STATS) {
    __syncthreads();
    float* fold = reinterpret_cast<float*>(lds);   // [NT][16]
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      fold[threadIdx.x * 16 + k] = s1[k];
      fold[threadIdx.x * 16 + 8 + k] = s2[k];
    }
    __syncthreads();
    constexpr int Q = NT / CPR;                    // threads sharing a column group
    for (int c = threadIdx.x; c < BN; c += NT) {
      const int gq = c / 8, k = c % 8;
      float a = 0.f, b = 0.f;
      for (int q = 0; q < Q; ++q) {               // fixed order: deterministic
        a += fold[(q * CPR + gq) * 16 + k];
        b += fold[(q * CPR + gq) * 16 + 8 + k];
      }
      stats[(int64_t)tm * 2 * Co + n0 + c] = a;
      stats[(int64_t)tm * 2 * Co + Co + n0 + c] = b;
    }
  }
}

bool conv3_tap_ok(int C, int Co, int H, int W) {
  if (C % 32 != 0 || C < 32 || (Co % 128 != 0 && Co != 64) || W < 4 || W > 224) return false;
  if (T3_M % W != 0) return false;
  const int R = T3_M / W;
  if ((R + 2) * (W + 2) * 64 > T3_PATCH) return false;
  return H >= 1;
}

int conv3_tap_bn(int Co) { return Co % 128 == 0 ? 128 : 64; }

int conv3_tap_tiles_m(int N, int H, int W) {
  const int R = T3_M / W;
  return (N * H + R - 1) / R;
}

void conv3_tap(const uint16_t* x, const uint16_t* w, uint16_t* y, float* stats, int N, int H,
               int W, int C, int Co, hipStream_t st) {
  const int NH = N * H;
  const int bn = conv3_tap_bn(Co);
  const int tiles = conv3_tap_tiles_m(N, H, W) * (Co / bn);
  const uint32_t xb = (uint32_t)((int64_t)NH * W * C * 2);
  const uint32_t wb = (uint32_t)((int64_t)Co * 9 * C * 2);
#define LW_T3(BNV, ST)                                                                             \
  hipLaunchKernelGGL((k_conv3_tap<BNV, ST>), dim3(tiles), dim3(BNV * 4), 0, st, x, w, y, stats,    \
                     NH, H, W, C, Co, xb, wb)
  if (bn == 128) {
    if (stats) LW_T3(128, true);
    else LW_T3(128, false);
  } else {
    if (stats) LW_T3(64, true);
    else LW_T3(64, false);
  }
#undef LW_T3
}

}  // namespace lw
