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
// LDS (per workgroup, 2 workgroups per CU): two 24 KB patch buffers (chunk c and c + 1) and a ring
// of 3 weight slices (K-steps s, s + 1, s + 2), all filled by LDS-DMA (buffer_load ... lds). Both
// are stored as 4 planes, one per 8-channel k group g: [g][pixel][16 B] (plane stride 6 KB) and
// [g][row][16 B] (plane stride BN·16 B). A ds_read_b128 is served per 16-lane group {0-3, 12-15,
// 20-27}, {4-11, 16-19, 28-31}, ... (MI355X_MICROARCH.md §LDS): its lanes are 16 consecutive
// pixels of two k groups whose planes start on a 256-byte boundary, so the 16 reads land in 16
// distinct bank quads for ANY first pixel — an interleaved [pixel][4 x 16 B] image with an XOR
// swizzle was 2-way conflicted at 14 of 16 start offsets (the taps shift the start).
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
constexpr int T3_PLANE = T3_PATCH / 4;    // bytes per 8-channel plane of a patch buffer
constexpr int T3_PBLK = T3_PLANE / 1024;  // 64-pixel DMA blocks per plane

// LW_T3_ZSEL: a tap's out-of-image fragment lanes read a zeroed 16-byte LDS slot instead of being
// zeroed after the read — one address select per fragment instead of four register selects (the
// tap kernels issue 6-10 VALU per MFMA: profiles/r6/pmc_conv3/). 2: also each fragment address
// is one add of the lane's hoisted byte base and the step's wave-uniform offset (kept opaque in
// an SGPR so the 63 (block, tap) addresses are not hoisted into registers), instead of a copy of
// the pixel index, a shift and an add.
#ifndef LW_T3_ZSEL
#define LW_T3_ZSEL 2
#endif
#ifndef LW_T3_PEN
#define LW_T3_PEN 1      // BN = 64: masked taps by max() with per-lane penalties (see below)
#endif

template <int N>
__device__ __forceinline__ void t3_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// BN output channels per workgroup (BN / 16 waves: 2 pixel halves x BN / 32 channel groups)
// DEPTH: weight slices in the ring (3: prefetch 2 K-steps ahead; 4: 3 ahead, 80 KB of LDS at
// BN = 128, still two workgroups per CU)
// TPB > 1: TPB taps (K-steps) per barrier, ring of 2·TPB weight slices (the next TPB prefetched
// while the current TPB are computed), one s_waitcnt vmcnt(0) + barrier per TPB steps.
template <int BN, bool STATS, int DEPTH = T3_NWS, int TPB = 1>
__global__ __launch_bounds__(BN * 4)
__attribute__((amdgpu_waves_per_eu(BN == 128 && 2 * T3_PATCH + DEPTH * BN * 64 <= 81920 ? 4 : 2)))
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
  constexpr int LDS = 2 * T3_PATCH + DEPTH * WSL;
  constexpr int AH = DEPTH - 1;                    // K-steps of weight prefetch
  constexpr int LDH = BN + 8;                      // bf16 staging row (epilogue)
  static_assert(T3_M * LDH * 2 <= LDS, "epilogue staging fits the ring");
  static_assert(NT * 16 * 4 <= LDS, "statistics fold fits");
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS + 16];   // + the zero slot
  if (LW_T3_ZSEL && threadIdx.x == 0)              // visible after the prologue's barrier
    *reinterpret_cast<uint4*>(lds + LDS) = make_uint4(0u, 0u, 0u, 0u);

  // patch pixel q <-> flat input pixel (g0 - 1) * W - 1 + q: rows g0-1 .. g0+R plus one pixel on
  // each side, no halo columns (a tap column outside the image is masked like a tap row)
  const int R = T3_M / W, npix = (R + 2) * W + 2;
  const int tiles_n = Co / BN;
  const int total = gridDim.x;
  const int pid = xcd_remap((int)blockIdx.x, total);   // the n-tiles of one m-tile share an XCD
  const int tm = pid / tiles_n, tn = pid - tm * tiles_n;
  const int g0 = tm * R;                          // first output row (global row space)
  const int n0 = tn * BN;
  const int NC = C / 32, S = 9 * NC;
  const int64_t K = 9 * (int64_t)C;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
  const int wm = wave & 1, wn = wave >> 1;        // pixel half (7 blocks), 32-channel group
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(x, x_bytes), rw = make_rsrc(w, w_bytes);

  // ---- per-thread DMA sources. Patch: global instruction I = j*NWAVE + wave fills plane
  // g = I / T3_PBLK (8-channel group g of the chunk), patch pixels (I % T3_PBLK)*64 + lane
  int prel[NPJ];                                   // flat pixel rel. to the patch's first
  uint32_t pok = 0;                                // inside the patch
#pragma unroll
  for (int j = 0; j < NPJ; ++j) {
    const int I = j * NWAVE + wave;
    const int gs = I / T3_PBLK, q = (I - gs * T3_PBLK) * 64 + l;
    prel[j] = q * C * 2 + gs * 16;
    pok |= (q < npix ? 1u : 0u) << j;
  }
  const int64_t P0 = (int64_t)(g0 - 1) * W - 1;   // flat pixel of patch pixel 0 (may be < 0)
  const int64_t NHW = (int64_t)NH * W;
  auto issue_patch = [&](int c, int buf) {
    uint8_t* dst = lds + buf * T3_PATCH;
#pragma unroll
    for (int j = 0; j < NPJ; ++j) {
      const int I = j * NWAVE + wave;
      const int q = (I - (I / T3_PBLK) * T3_PBLK) * 64 + l;
      const int64_t P = P0 + q;
      const bool ok = ((pok >> j) & 1u) && P >= 0 && P < NHW;
      const uint32_t off = ok ? (uint32_t)(P0 * C * 2) + (uint32_t)prel[j] + (uint32_t)(c * 64)
                              : OOB;
      glds16(rx, reinterpret_cast<uint16_t*>(dst + I * 1024), off);
    }
  };
  // weight slice of K-step s = (c, t): plane g = wave / (BN/64) (k = t*C + c*32 + 8g), rows
  // (wave % (BN/64))*64 + lane
  const int wg = wave / (BN / 64), wrow = (wave - wg * (BN / 64)) * 64 + l;
  const uint32_t wrel = (uint32_t)(((int64_t)(n0 + wrow) * K + wg * 8) * 2);
  auto issue_w = [&](int s, int slot) {
    const int c = s / 9, t = s - c * 9;
    uint32_t wr = wrel;
    asm volatile("" : "+v"(wr));                   // (not hoisted per step: registers)
    const uint32_t off = wr + (uint32_t)((t * C + c * 32) * 2);
    glds16(rw, reinterpret_cast<uint16_t*>(lds + 2 * T3_PATCH + slot * WSL + wave * 1024), off);
  };

  // ---- per-lane fragment geometry: pixel blocks wm*7 + i, lane pixel (l & 15); k group g
  const int g = l >> 4;
  int ppix[7];                 // patch pixel of tap (0, 0): m + (row 0) - 1 + 1
  uint32_t vmask = 0;          // per block i, 4 bits: tap row 0 / row 2 / col 0 / col 2 inside
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int m = (wm * 7 + i) * 16 + (l & 15);
    const int orow = m / W, ox = m - orow * W;
    ppix[i] = m;
    const int yy = (g0 + orow) % H;
    vmask |= (yy >= 1 ? 1u : 0u) << (4 * i);
    vmask |= (yy + 1 < H ? 1u : 0u) << (4 * i + 1);
    vmask |= (ox >= 1 ? 1u : 0u) << (4 * i + 2);
    vmask |= (ox + 1 < W ? 1u : 0u) << (4 * i + 3);
  }
  const int pplane = g * T3_PLANE;                 // this lane's k group: its patch plane
  uint32_t pbyte[7];                               // ZSEL 2: byte of patch pixel ppix[i], plane g
#pragma unroll
  for (int i = 0; i < 7; ++i) pbyte[i] = (uint32_t)(pplane + ppix[i] * 16);
  // BN = 64 (registers to spare at two waves per SIMD): a masked tap's address is
  // max(address, row penalty, column penalty) — one v_max3 — where a penalty is the zero slot's
  // address (above every patch address) for an out-of-image tap row / column, else 0
  constexpr bool PEN = LW_T3_ZSEL >= 2 && LW_T3_PEN && BN == 64;
  uint32_t rpen[2][PEN ? 7 : 1], cpen[2][PEN ? 7 : 1];
#pragma unroll
  for (int i = 0; i < (PEN ? 7 : 1); ++i) {
    rpen[0][i] = ((vmask >> (4 * i)) & 1u) ? 0u : (uint32_t)LDS;
    rpen[1][i] = ((vmask >> (4 * i)) & 2u) ? 0u : (uint32_t)LDS;
    cpen[0][i] = ((vmask >> (4 * i)) & 4u) ? 0u : (uint32_t)LDS;
    cpen[1][i] = ((vmask >> (4 * i)) & 8u) ? 0u : (uint32_t)LDS;
  }
  int wbyte[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) wbyte[j] = (g * BN + wn * 32 + j * 16 + (l & 15)) * 16;

  f32x4 acc[7][2];
#pragma unroll
  for (int i = 0; i < 7; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const uint8_t* P, const uint8_t* Wt, int r, int s) {
    h16x8 fb[2], fa[7];
#pragma unroll
    for (int j = 0; j < 2; ++j) fb[j] = *reinterpret_cast<const h16x8*>(Wt + wbyte[j]);
    const int toff = r * W + s;
    if constexpr (LW_T3_ZSEL >= 2) {
      uint32_t uo = (uint32_t)(P - lds) + (uint32_t)(toff * 16);
      asm volatile("" : "+s"(uo));
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        const uint32_t a = pbyte[i] + uo;
        if (PEN && (r != 1 || s != 1)) {
          const uint32_t rp = r == 1 ? 0u : rpen[r >> 1][i], cp = s == 1 ? 0u : cpen[s >> 1][i];
          fa[i] = *reinterpret_cast<const h16x8*>(lds + max(max(a, rp), cp));
        } else if (r != 1 || s != 1) {
          const uint32_t need = (r == 0 ? 1u : r == 2 ? 2u : 0u) | (s == 0 ? 4u : s == 2 ? 8u : 0u);
          const bool ok = ((vmask >> (4 * i)) & need) == need;
          fa[i] = *reinterpret_cast<const h16x8*>(lds + (ok ? a : (uint32_t)LDS));
        } else {
          fa[i] = *reinterpret_cast<const h16x8*>(lds + a);
        }
      }
    } else {
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      // opaque base: keeps the 63 (block, tap) addresses from being hoisted out of the K loop
      // into registers (they would spill)
      int pb = ppix[i];
      asm volatile("" : "+v"(pb));
      const int p = pb + toff;
      if (r != 1 || s != 1) {
        const uint32_t need = (r == 0 ? 1u : r == 2 ? 2u : 0u) | (s == 0 ? 4u : s == 2 ? 8u : 0u);
        const bool ok = ((vmask >> (4 * i)) & need) == need;
        if (LW_T3_ZSEL) {
          fa[i] = *reinterpret_cast<const h16x8*>(ok ? P + pplane + p * 16 : lds + LDS);
        } else {
          fa[i] = *reinterpret_cast<const h16x8*>(P + pplane + p * 16);
          if (!ok) fa[i] = h16x8{};
        }
      } else {
        fa[i] = *reinterpret_cast<const h16x8*>(P + pplane + p * 16);
      }
    }
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 7; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = mfma16(fb[j], fa[i], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
  };

  if constexpr (TPB > 1) {
    static_assert(DEPTH == 2 * TPB, "ring of two super-steps");
    issue_patch(0, 0);
#pragma unroll
    for (int q = 0; q < TPB; ++q) issue_w(q, q);
    t3_wait_barrier<0>();
#pragma unroll 1
    for (int base = 0; base < S; base += TPB) {
      const int half = (base / TPB) & 1;             // ring half holding this super-step
#pragma unroll
      for (int q = 0; q < TPB; ++q)
        if (base + TPB + q < S) issue_w(base + TPB + q, (half ^ 1) * TPB + q);
#pragma unroll
      for (int q = 0; q < TPB; ++q) {
        const int s2 = base + q, c2 = s2 / 9;
        if (s2 < S && s2 - c2 * 9 == 4 && c2 + 1 < NC) issue_patch(c2 + 1, (c2 + 1) & 1);
      }
#pragma unroll
      for (int q = 0; q < TPB; ++q) {
        const int s2 = base + q;
        if (s2 < S) {
          const int c2 = s2 / 9, t2 = s2 - c2 * 9;
          compute(lds + (c2 & 1) * T3_PATCH, lds + 2 * T3_PATCH + (half * TPB + q) * WSL, t2 / 3,
                  t2 % 3);
        }
      }
      t3_wait_barrier<0>();
    }
  } else {
  // ---- prologue: patch of chunk 0, weight slices 0 .. AH-1 (S >= 9 > AH)
  issue_patch(0, 0);
#pragma unroll
  for (int q = 0; q < AH; ++q) issue_w(q, q);
  t3_wait_barrier<AH - 1>();                       // slice 0 and the patch landed
  int slot = 0;
#pragma unroll 1
  for (int c = 0; c < NC; ++c) {
    const uint8_t* P = lds + (c & 1) * T3_PATCH;
    const bool next_chunk = c + 1 < NC;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int s = c * 9 + t;
      // slice s + AH goes to the slot read at step s - 1 (retired by that step's barrier)
      if (s + AH < S) issue_w(s + AH, slot == 0 ? DEPTH - 1 : slot - 1);
      if (t == 4 && next_chunk) issue_patch(c + 1, (c + 1) & 1);
      compute(P, lds + 2 * T3_PATCH + slot * WSL, t / 3, t % 3);
      // wait for slice s + 1 only: the DMAs issued after it (later slices, and the next
      // chunk's patch when it was issued within the last AH steps) may stay in flight
      const int later = (s + 2 < S ? 1 : 0) + (AH >= 3 && s + 3 < S ? 1 : 0);
      const bool pend = next_chunk && t >= 4 && t < 4 + AH;
      if (pend) {
        if (later == 2) t3_wait_barrier<NPJ + 2>();
        else if (later == 1) t3_wait_barrier<NPJ + 1>();
        else t3_wait_barrier<NPJ>();
      } else {
        if (later == 2) t3_wait_barrier<2>();
        else if (later == 1) t3_wait_barrier<1>();
        else t3_wait_barrier<0>();
      }
      slot = slot == DEPTH - 1 ? 0 : slot + 1;
    }
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
      for (int r = 0; r < 4; ++r) h[r] = f2h(acc[i][j][r]);
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
        const float f = k & 1 ? hhi(u[k >> 1]) : hlo(u[k >> 1]);
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
  if (((R + 2) * W + 2) * 64 > T3_PATCH) return false;     // (the wgrad's patch: the same)
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
  // a ring of 3 slices with one barrier per tap (rings of 4 / 6 slices with 1 / 2 / 3 taps per
  // barrier measured no faster and were removed in round 6)
#define LW_T3(BNV, ST, D, T)                                                                       \
  hipLaunchKernelGGL((k_conv3_tap<BNV, ST, D, T>), dim3(tiles), dim3(BNV * 4), 0, st, x, w, y,      \
                     stats, NH, H, W, C, Co, xb, wb)
#define LW_T3V(D, T)                                                                               \
  do {                                                                                             \
    if (bn == 128) {                                                                               \
      if (stats) LW_T3(128, true, D, T);                                                           \
      else LW_T3(128, false, D, T);                                                                \
    } else {                                                                                       \
      if (stats) LW_T3(64, true, D, T);                                                            \
      else LW_T3(64, false, D, T);                                                                 \
    }                                                                                              \
  } while (0)
  LW_T3V(3, 1);
#undef LW_T3V
#undef LW_T3
}

}  // namespace lw

namespace lw {

// ---------------------------------------------------------------------------------------------
// Weight gradient of the same convolution: dW[co][r][s][ci] = Σ_p dy[p][co] · x[p + (r-1, s-1)][ci].
// A workgroup owns a (BM output channels) x (9 taps x 32 input channels) block of dW and a
// contiguous range of 224-pixel tiles (the reduction over pixels is split over workgroups; one
// fp32 slab per split, summed in fixed order by k_conv3_tap_reduce). Per tile the x patch of its
// 32-channel chunk is staged once (as in the forward) and read by all 9 taps; dy streams through
// a ring of 32-pixel slices [32 px][BM co]. Both MFMA operands have the pixel as their k index,
// so both are read with the transposing ds_read_b64_tr_b16 (cdna_hip_programming.md T10):
//   dy slice: 16-byte chunk c of row r at c ^ X(r) (X(r) = ((r & 3) << 2) | ((r >> 2) & 3) for
//             256-byte rows; a pair-level XOR for 128-byte rows), the two 8-row blocks a 32-lane
//             half reads hitting disjoint banks;
//   x patch:  the forward's halo-free pixel order in 4 planes, plane stride ≡ 64 (mod 256) bytes
//             (conflict-free for the 8 rows x 2 planes a 32-lane half reads); a tap outside the
//             pixel's image reads a zero row instead (the read gathers across lanes: pad, don't mask).
// Waves: BM / 32 channel pairs x 2 halves of the 18 (tap, 16-channel) column blocks; 2 x 9 MFMAs
// per wave and 32-pixel k-step.
constexpr int T3W_KS = T3_M / 32;          // 32-pixel k-steps per tile

template <int BM>
__device__ __forceinline__ int t3w_dy_chunk(int r, int c) {
  if constexpr (BM == 128) return c ^ (((r & 3) << 2) | ((r >> 2) & 3));
  else return c ^ ((((r >> 1) & 1) | (((r >> 3) & 1) << 1)) << 1);
}

constexpr int T3W_PLANE = 6208;           // patch plane stride of the weight gradient (≡ 64 mod 256)
constexpr int T3W_PATCH = 4 * T3W_PLANE;

template <int BM>
__global__ __launch_bounds__(BM * 4) __attribute__((amdgpu_waves_per_eu(2)))
void k_conv3_tap_wgrad(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
                       float* __restrict__ part, int NH, int H, int W, int C, int Co,
                       int tiles_p, int tps, uint32_t dy_bytes, uint32_t x_bytes) {
  constexpr int NWAVE = BM / 16;
  constexpr int NPJ = 24 / NWAVE;                   // 4 planes x 6 blocks of 64 pixels
  constexpr int DSL = 32 * BM * 2;                  // bytes per dy slice
  constexpr int LDS = 2 * T3W_PATCH + T3_NWS * DSL + 64;
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS];
  uint8_t* zero_row = lds + 2 * T3W_PATCH + T3_NWS * DSL;

  const int out_tiles = (Co / BM) * (C / 32);
  const int ot = (int)blockIdx.x % out_tiles, split = (int)blockIdx.x / out_tiles;
  const int co0 = (ot / (C / 32)) * BM, cc = ot % (C / 32), ci0 = cc * 32;
  const int tp0 = split * tps, tp1 = min(tp0 + tps, tiles_p);
  const int ntiles = tp1 - tp0;
  const int R = T3_M / W, npix = (R + 2) * W + 2;
  const int64_t NHW = (int64_t)NH * W;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
  const int cw = wave % (BM / 32), nh = wave / (BM / 32);
  const __amdgpu_buffer_rsrc_t rd = make_rsrc(dy, dy_bytes), rx = make_rsrc(x, x_bytes);
  if (threadIdx.x < 4) reinterpret_cast<uint4*>(zero_row)[threadIdx.x] = make_uint4(0u, 0u, 0u, 0u);

  // ---- patch DMA (the forward's halo-free pixel order, plane stride T3W_PLANE), chunk cc
  int prel[NPJ], pq[NPJ], pdst[NPJ];
#pragma unroll
  for (int j = 0; j < NPJ; ++j) {
    const int I = j * NWAVE + wave;
    const int gs = I / 6, q = (I - gs * 6) * 64 + l;
    pq[j] = q;
    prel[j] = q * C * 2 + gs * 16;
    pdst[j] = gs * T3W_PLANE + (I - gs * 6) * 1024;
  }
  auto issue_patch = [&](int u, int buf) {
    const int g0 = (tp0 + u) * R;
    const int64_t P0 = (int64_t)(g0 - 1) * W - 1;
    const uint32_t base = (uint32_t)(P0 * C * 2) + (uint32_t)(cc * 64);
    uint8_t* dst = lds + buf * T3W_PATCH;
#pragma unroll
    for (int j = 0; j < NPJ; ++j) {
      const int64_t P = P0 + pq[j];
      const bool ok = pq[j] < npix && P >= 0 && P < NHW;
      glds16(rx, reinterpret_cast<uint16_t*>(dst + pdst[j]), ok ? base + (uint32_t)prel[j] : OOB);
    }
  };
  // ---- dy slice DMA: lane lands at row (wave*1024 + 16*l) / (2*BM), physical chunk -> logical
  const int drow = (wave * 1024 + 16 * l) / (2 * BM);
  const int dch = t3w_dy_chunk<BM>(drow, (16 * l) % (2 * BM) / 16);
  auto issue_dy = [&](int s, int slot) {
    const int u = s / T3W_KS, ks = s - u * T3W_KS;
    const int64_t p = (int64_t)(tp0 + u) * T3_M + ks * 32 + drow;
    const uint32_t off = p < NHW ? (uint32_t)((p * Co + co0 + dch * 8) * 2) : OOB;
    glds16(rd, reinterpret_cast<uint16_t*>(lds + 2 * T3W_PATCH + slot * DSL + wave * 1024), off);
  };

  // ---- per-lane transposed-read geometry: group g, row q, 4-column block p4
  const int g = l >> 4, q4 = (l & 15) >> 2, p4 = l & 3;
  // dy (A operand) byte offsets within a slice for rows 8g + q (+4), channel blocks 2cw, 2cw + 1
  int aoff[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int rr = 8 * g + q4 + 4 * hh;
      const int col = (2 * cw + i) * 16 + 4 * p4;
      aoff[i][hh] = rr * (2 * BM) + t3w_dy_chunk<BM>(rr, col >> 3) * 16 + (col & 7) * 2;
    }

  f32x4 acc[2][9];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  typedef __attribute__((address_space(3))) i16x4 lds_v4;
  auto tr = [&](const uint8_t* a) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)a); };
  auto cat8 = [](i16x4 lo, i16x4 hi) {
    typedef short i16x8 __attribute__((ext_vector_type(8)));
    const i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(h16x8, v);
  };
  auto compute = [&](const uint8_t* P, const uint8_t* D, int g0, int ks) {
    h16x8 fa[2], fb[9];
#pragma unroll
    for (int i = 0; i < 2; ++i) fa[i] = cat8(tr(D + aoff[i][0]), tr(D + aoff[i][1]));
    // this lane's two rows: pixels m = ks*32 + 8g + q4 (+4) of the tile, patch pixel m + tap
    int mm[2];
    uint32_t vm = 0;           // per row: tap row 0 / row 2 / col 0 / col 2 inside the image
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      int m = ks * 32 + 8 * g + q4 + 4 * hh;
      asm volatile("" : "+v"(m));
      const int orow = m / W, ox = m - orow * W, yy = (g0 + orow) % H;
      mm[hh] = m;
      vm |= ((yy >= 1 ? 1u : 0u) | (yy + 1 < H ? 2u : 0u) | (ox >= 1 ? 4u : 0u) |
             (ox + 1 < W ? 8u : 0u)) << (4 * hh);
    }
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int nb = nh * 9 + j, t = nb >> 1, hc = nb & 1;
      const int r = t / 3, s = t - r * 3;
      const uint32_t need = (r == 0 ? 1u : r == 2 ? 2u : 0u) | (s == 0 ? 4u : s == 2 ? 8u : 0u);
      const int plane = (2 * hc + (p4 >> 1)) * T3W_PLANE, wb = (p4 & 1) * 8;
      const uint8_t* a[2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int q = mm[hh] + r * W + s;
        const bool ok = ((vm >> (4 * hh)) & need) == need;
        a[hh] = ok ? P + plane + q * 16 + wb : zero_row + wb;
      }
      fb[j] = cat8(tr(a[0]), tr(a[1]));
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 9; ++j)
        acc[i][j] = mfma16(fb[j], fa[i], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
  };

  const int S = ntiles * T3W_KS;
  if (S > 0) {
    issue_patch(0, 0);
    issue_dy(0, 0);
    if (S > 1) issue_dy(1, 1);
    if (S > 1) t3_wait_barrier<1>();
    else t3_wait_barrier<0>();
    int slot = 0;
#pragma unroll 1
    for (int u = 0; u < ntiles; ++u) {
      const uint8_t* P = lds + (u & 1) * T3W_PATCH;
      const bool next_tile = u + 1 < ntiles;
      const int g0 = (tp0 + u) * R;
#pragma unroll
      for (int ks = 0; ks < T3W_KS; ++ks) {
        const int s = u * T3W_KS + ks;
        const bool w2 = s + 2 < S;
        if (w2) issue_dy(s + 2, slot == 0 ? 2 : slot - 1);
        if (ks == 3 && next_tile) issue_patch(u + 1, (u + 1) & 1);
        compute(P, lds + 2 * T3W_PATCH + slot * DSL, g0, ks);
        if ((ks == 3 || ks == 4) && next_tile) {
          if (w2) t3_wait_barrier<NPJ + 1>();
          else t3_wait_barrier<NPJ>();
        } else {
          if (w2) t3_wait_barrier<1>();
          else t3_wait_barrier<0>();
        }
        slot = slot == 2 ? 0 : slot + 1;
      }
    }
  }
  // ---- this split's slab: lane holds dW[co = block row (l & 15)][n = 4g + r] of each block
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int nb = nh * 9 + j, t = nb >> 1, hc = nb & 1;
      const int co = co0 + (2 * cw + i) * 16 + (l & 15);
      const int ci = ci0 + hc * 16 + 4 * g;
      *reinterpret_cast<float4*>(part + (((int64_t)split * Co + co) * 9 + t) * C + ci) =
          make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
}

// out[i] (+)= Σ_z part[z][i], z in order (deterministic), float4 per thread
__global__ __launch_bounds__(256) void k_conv3_tap_reduce(const float* __restrict__ part,
                                                          float* __restrict__ out, int64_t n4,
                                                          int zs, int accumulate) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 a = accumulate ? reinterpret_cast<const float4*>(out)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    for (int z = 0; z < zs; ++z) {
      const float4 v = reinterpret_cast<const float4*>(part)[(int64_t)z * n4 + i];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    reinterpret_cast<float4*>(out)[i] = a;
  }
}

int conv3_tap_wgrad_splits(int N, int H, int W, int C, int Co) {
  const int bm = Co % 128 == 0 ? 128 : 64;
  const int out_tiles = (Co / bm) * (C / 32);
  const int tiles_p = conv3_tap_tiles_m(N, H, W);
  // 8 waves per CU at 256 VGPRs: one 8-wave (BM 128) or two 4-wave (BM 64) workgroups per CU
  int splits = std::max(1, (bm == 64 ? 2 : 1) * cu_count() / out_tiles);
  splits = std::min(splits, tiles_p);
  const int tps = (tiles_p + splits - 1) / splits;
  return (tiles_p + tps - 1) / tps;
}

void conv3_tap_wgrad(const uint16_t* dy, const uint16_t* x, float* part, float* out, int N,
                     int H, int W, int C, int Co, int accumulate, hipStream_t st) {
  const int NH = N * H;
  const int bm = Co % 128 == 0 ? 128 : 64;
  const int out_tiles = (Co / bm) * (C / 32);
  const int tiles_p = conv3_tap_tiles_m(N, H, W);
  const int splits = conv3_tap_wgrad_splits(N, H, W, C, Co);
  const int tps = (tiles_p + splits - 1) / splits;
  const uint32_t dyb = (uint32_t)((int64_t)NH * W * Co * 2);
  const uint32_t xb = (uint32_t)((int64_t)NH * W * C * 2);
  const dim3 grid((unsigned)(out_tiles * splits));
  if (bm == 128)
    hipLaunchKernelGGL((k_conv3_tap_wgrad<128>), grid, dim3(512), 0, st, dy, x, part, NH, H, W,
                       C, Co, tiles_p, tps, dyb, xb);
  else
    hipLaunchKernelGGL((k_conv3_tap_wgrad<64>), grid, dim3(256), 0, st, dy, x, part, NH, H, W, C,
                       Co, tiles_p, tps, dyb, xb);
  const int64_t n4 = (int64_t)Co * 9 * C / 4;
  int64_t blocks = (n4 + 255) / 256;
  blocks = std::min<int64_t>(blocks, 4 * cu_count());
  hipLaunchKernelGGL(k_conv3_tap_reduce, dim3((unsigned)blocks), dim3(256), 0, st, part, out, n4,
                     splits, accumulate);
}

}  // namespace lw
