// Large-tile bf16 MFMA GEMM for gfx950: 256x256 (or 256x128) output tile per 512-thread workgroup
// (8 waves as 2 (M) x 4 (N), each wave 128x64), BK = 64. Operands K-contiguous (A [M][K], B [N][K]:
// x·Wᵀ of a Linear / 1x1 convolution, the square benchmark shapes), both M/N-contiguous (weight
// gradients dYᵀ·X), or a K-contiguous A with an N-contiguous B (data gradients dY·W).
//
// Why a second GEMM structure: the 128x128 / 4-wave tiles of gemm_core.h cross a workgroup barrier
// with vmcnt(0) once per K-step, which caps them near 900 TFLOP/s on large problems
// (profiles/r2_gemm_tile_experiments.txt: 8192^3 at 0.84-1.05 PF vs hipBLASLt 1.45-1.57). Here the
// LDS-DMA prefetch stays in flight across the barriers (cdna_hip_programming.md §5 "256² 8-phase
// template"):
//   * LDS = 2 buffers x 4 half-tiles of 16 KB (A rows of quadrant row 0 / 1, B cols of quadrant
//     col 0 / 1), filled by buffer_load ... lds (16 B per lane, XOR-swizzled on the SOURCE address
//     so the lane-linear LDS image is bank-conflict free for ds_read_b128);
//   * each K-tile is computed in 4 phases, one 64x32 C-quadrant per wave per phase
//     (16 x v_mfma_f32_16x16x32_bf16). A phase is  R: ds_reads + one half-tile DMA + counted waits
//     | barrier | M: the MFMA cluster (s_setprio 1) | barrier;
//   * the two wave rows run staggered by one barrier (row 1 takes an extra barrier up front), so on
//     every SIMD one wave reads LDS / issues DMA while its partner runs MFMAs;
//   * a half-tile is refilled for a later K-tile one phase after its last read (the reads are
//     retired by lgkmcnt(0) before the barrier that ends R, so with the stagger both rows are past
//     them), and five half-tiles stay in flight: every load gets 6-7 phases to land;
//   * one `s_waitcnt vmcnt(10)` (5 half-tiles x 2 loads) at the end of R in P0, P1, P3 retires the
//     data read in the next phase; raw s_barrier only (a __syncthreads() would drain every DMA).
// Issue order in K-tile c (buffer c&1; halves A0/A1 = A rows of quadrant row 0/1, B0/B1 = B cols):
//   P0: read A0,B0 -> Q00   DMA (c+1).A1 -> buffer (c+1)&1   vmcnt: (c).B1 landed
//   P1: read B1    -> Q01   DMA (c+2).A0 -> buffer c&1       vmcnt: (c).A1 landed
//   P2: read A1    -> Q11   DMA (c+2).B0 -> buffer c&1
//   P3: (registers)-> Q10   DMA (c+2).B1 -> buffer c&1       vmcnt: (c+1).A0,B0 landed
// Epilogues: bf16 / fp32 store with bias + ReLU (+ column statistics, one row per wave row), or
// an fp32 split-K slab (reduced by k_splitk_reduce in gemm.hip, fixed order).
// GA: the A operand is the im2col row gather of a convolution (conv.hip CV_A, one parity class,
// C % 64 == 0): a K-tile then lies inside one filter tap, so a lane's DMA source is its pixel's
// window origin + the tap's (uniform) offset, and a tap falling into the padding becomes an OOB
// offset (the DMA lands zeros) — the same big-tile schedule runs the 3x3 forward and stride-1
// data-gradient convolutions with no im2col buffer. GB: the B operand of a weight gradient is the
// im2col column gather (column = (tap, channel), row = output pixel, decoded per K-tile).
#include "common.h"
#include "gemm_core.h"

namespace lw {

constexpr int BGT = 512;                     // threads
constexpr int BBM = 256, BBK = 64;
constexpr int AHALF = 128 * BBK;             // bf16 elements per A half-tile (16 KB)

// element offset of 16-byte chunk c of stored row r in a half-tile (128-byte rows, XOR swizzle)
__device__ __forceinline__ int big_off(int r, int c) { return r * BBK + ((c ^ (r & 7)) << 3); }

// MN-contiguous operands (A [K][M], B [K][N]: a weight gradient dYᵀ·X) are staged as [k][column]
// images of W = 128 or 64 columns and read by ds_read_b64_tr_b16 (the transposing LDS read): a
// lane reads 8 bytes at row k = 32s + 8g + q (+4) and columns i + 4p (gemm_core.h load_frag). The
// 16-byte chunk of column c in row k is stored at chunk (c/8) ^ x(k), which puts the 8 rows one
// 32-lane group reads on 8 disjoint 32-byte windows of the bank row (conflict-free); the DMA
// swizzles its SOURCE address to match, the LDS image stays lane-linear.
__device__ __forceinline__ int xw128(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }
__device__ __forceinline__ int xw64(int k) { return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1)); }
template <int W>
__device__ __forceinline__ h16x8 frag_tr(const uint16_t* img, int i_base, int s) {
  const int l = threadIdx.x & 63;
  const int g = l >> 4, t = l & 15, q = t >> 2, p4 = t & 3;
  const int k0 = 32 * s + 8 * g + q;
  const int c = i_base + 4 * p4;
  const int x = W == 128 ? xw128(k0) : xw64(k0);       // the same for row k0 + 4
  const uint16_t* p0 = img + k0 * W + ((((c >> 3) ^ x) << 3) | (c & 7));
  typedef __attribute__((address_space(3))) i16x4 lds_v4;
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(p0));
  const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(p0 + 4 * W));
  typedef short i16x8 __attribute__((ext_vector_type(8)));
  const i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(h16x8, v);
}

template <int N>
__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// BN = 256 (wave tile 128x64) or 128 (wave tile 128x32); waves 2 (M) x 4 (N)
// (Tried: reading the next K-tile's B0 fragments in P3 after a wait moved to P2, so the LDS reads
// spread 8/4/8/4 over the phases instead of 12/4/8/0: 251 VGPRs and 7 % slower at 8192^3,
// profiles/r3/gemm_big_pf_ab.jsonl.)
// MN: A is MN-contiguous ([K][M]); MNB (default MN): B is ([K][N]). Mixed layouts (K-contiguous
// A with an N-contiguous B: a data gradient dY·W with W as stored) stage each operand its own way.
template <int BN, int EPI, bool MN, bool GA = false, bool GB = false, bool MNB = MN>
__global__ __launch_bounds__(BGT) void k_gemm_big(const GemmK p) {
  static_assert(!(GA && MN), "the row gather stages a K-contiguous A");
  static_assert(!GB || MNB, "the column gather (weight gradient) stages an MN-contiguous B");
  constexpr int BHALF = (BN / 2) * BBK;        // bf16 elements per B half-tile
  constexpr int BUF = 2 * AHALF + 2 * BHALF;   // one K-tile: A0 A1 B0 B1
  constexpr int NB = BN / 128;                 // DMA instructions per B half (A: 2)
  constexpr int QN = BN / 8;                   // columns of a wave's B quadrant
  constexpr int FQ = QN / 16;                  // 16-wide MFMA blocks per B quadrant
  // counted waits (loads issued after the half-tile the next phase reads; see the schedule)
  constexpr int VM_P01 = 3 * 2 + 2 * NB, VM_P3 = 2 * 2 + 3 * NB;
  static_assert(BN == 256 || BN == 128, "tile width");
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * BUF];   // one array (rule 4a)
  const int tiles_n = (p.N + BN - 1) / BN, tiles_m = (p.M + BBM - 1) / BBM;
  int tm, tn;
  int split;
  tile_split_of(tiles_m, tiles_n, tm, tn, split);     // gemm_core.h (split-K slices per XCD)
  const int m0 = tm * BBM, n0 = tn * BN;
  const int kbeg = split * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int T = kbeg < kend ? (kend - kbeg + BBK - 1) / BBK : 0;
  const int klen = kend - kbeg;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
  const int wm = w >> 2, wn = w & 3;   // wave-uniform (scalar): the stagger branch is a real branch

  // ---- per-thread DMA sources: A half qa (rows), instruction hh; B half qb (cols), instruction hb.
  // A row-chunk out of range → OOB (the buffer load returns zeros); the offset stays OOB when a
  // K-step is added (every operand is < 2 GiB)
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, p.a_bytes), rb = make_rsrc(p.B, p.b_bytes);
  uint32_t va[2][2], vb[2][NB];
  int ka[2], kb[NB];                   // k offset of the lane's chunk within a K-tile
  constexpr int WB = BN / 2;           // MN: columns of a B half image
  // GA: the pixel's window origin (hb, wb; rows past M fail every bounds test) and the byte offset
  // of its tap-(0, 0) chunk, per A half qa and instruction hh
  int ghb[2][2], gwb[2][2], grow[2][2];
  const int gC = p.cv.C, gHin = p.cv.Hin, gWin = p.cv.Win;
  const float inv_c = 1.f / (float)gC, inv_ts = 1.f / (float)p.cv.cls[0].TS;
  // GB (weight gradient): B rows are output pixels, columns (tap, channel) of the input window:
  // per B chunk the tap's window offset (bho, bwo; columns past N fail every bounds test) and,
  // in vb, the byte offset of (tap, channel) relative to the pixel's window origin
  int bho[2][NB], bwo[2][NB];
  const int gHw = p.cv.cls[0].Hg * p.cv.cls[0].Wg;
  const float inv_hw = 1.f / (float)gHw, inv_wg = 1.f / (float)p.cv.cls[0].Wg;
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const int q = threadIdx.x + hh * BGT;           // chunk of the half-tile this lane lands in
    if constexpr (GA) {
      const int lr = q >> 3, cc = q & 7;
      const int gc = cc ^ (lr & 7);
      ka[hh] = gc * 8;
      const ConvClass& k0c = p.cv.cls[0];
      const int hw = k0c.Hg * k0c.Wg;
#pragma unroll
      for (int qa = 0; qa < 2; ++qa) {
        const int row = m0 + (lr >> 6) * 128 + qa * 64 + (lr & 63);
        const bool in = row < k0c.M;
        const int mm = in ? row : 0;
        const int b = mm / hw, rem = mm - b * hw;
        const int y = rem / k0c.Wg, x = rem - y * k0c.Wg;
        const int h0 = y * p.cv.sh + k0c.oh, w0 = x * p.cv.sw + k0c.ow;
        ghb[qa][hh] = in ? h0 : -(1 << 28);
        gwb[qa][hh] = w0;
        grow[qa][hh] = (((b * gHin + h0) * gWin + w0) * gC + gc * 8) * 2;
        va[qa][hh] = 0;
      }
    } else if constexpr (!MN) {
      const int lr = q >> 3, cc = q & 7;
      const int gc = cc ^ (lr & 7);                 // logical chunk fetched (swizzle at the source)
      ka[hh] = gc * 8;
#pragma unroll
      for (int qa = 0; qa < 2; ++qa) {
        const int row = m0 + (lr >> 6) * 128 + qa * 64 + (lr & 63);
        va[qa][hh] = row < p.M ? (uint32_t)(((int64_t)row * p.lda + kbeg + gc * 8) * 2) : OOB;
      }
    } else {
      const int k = q >> 4, lc = (q & 15) ^ xw128(k);   // [64 k][128 m] image
      ka[hh] = k;
#pragma unroll
      for (int qa = 0; qa < 2; ++qa) {
        const int m = m0 + (lc >> 3) * 128 + qa * 64 + (lc & 7) * 8;
        va[qa][hh] = m < p.M ? (uint32_t)(((int64_t)(kbeg + k) * p.lda + m) * 2) : OOB;
      }
    }
  }
#pragma unroll
  for (int hb = 0; hb < NB; ++hb) {
    const int q = threadIdx.x + hb * BGT;
    if constexpr (!MNB) {
      const int lr = q >> 3, cc = q & 7;
      const int gc = cc ^ (lr & 7);
      kb[hb] = gc * 8;
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        const int col = n0 + (lr / QN) * (BN / 4) + qb * QN + (lr % QN);
        vb[qb][hb] = col < p.N ? (uint32_t)(((int64_t)col * p.ldb + kbeg + gc * 8) * 2) : OOB;
      }
    } else {
      const int k = q / (WB / 8);
      const int lc = (q % (WB / 8)) ^ (WB == 128 ? xw128(k) : xw64(k));
      kb[hb] = k;
      const int c = lc * 8;
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        const int n = n0 + (c / QN) * (BN / 4) + qb * QN + (c % QN);
        if constexpr (GB) {
          // column n = (tap, channel): the chunk's window offset, fixed for the kernel
          const int nn = n < p.N ? n : 0;
          int ci;
          const int t = fdivmod(nn, gC, inv_c, ci);
          int js;
          const int jr = fdivmod(t, p.cv.cls[0].TS, inv_ts, js);
          const int ho = p.cv.cls[0].oh + p.cv.dh * jr;
          bwo[qb][hb] = p.cv.cls[0].ow + p.cv.dw * js;
          vb[qb][hb] = (uint32_t)(((ho * gWin + bwo[qb][hb]) * gC + ci) * 2);
          bho[qb][hb] = n < p.N ? ho : -(1 << 28);
        } else {
          vb[qb][hb] = n < p.N ? (uint32_t)(((int64_t)(kbeg + k) * p.ldb + n) * 2) : OOB;
        }
      }
    }
  }
  // half h of K-tile kt into buffer buf: 0/1 = A quadrant row 0/1, 2/3 = B quadrant col 0/1.
  // Chunks past the K range are zero-filled (split-K slices and ragged K); K-tiles past the last
  // are never read, so their chunks only need to stay inside the operands.
  auto dma = [&](int kt, int buf, int h) {
    if (h < 2) {
      uint16_t* base = lds + buf * BUF + h * AHALF;
      if constexpr (GA) {
        // the K-tile's tap (jr, js) and first channel: uniform, exact float division (< 2^24)
        const int kk = kbeg + kt * BBK;
        int ci0;
        const int t = fdivmod(kk, gC, inv_c, ci0);
        int js;
        const int jr = fdivmod(t, p.cv.cls[0].TS, inv_ts, js);
        const int ho = p.cv.dh * jr, wo = p.cv.dw * js;
        const int delta = ((ho * gWin + wo) * gC + ci0) * 2;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const bool ok = kt * BBK + ka[hh] < klen &&
                          (unsigned)(ghb[h][hh] + ho) < (unsigned)gHin &&
                          (unsigned)(gwb[h][hh] + wo) < (unsigned)gWin;
          glds16(ra, base + (w * 64 + hh * BGT) * 8, ok ? (uint32_t)(grow[h][hh] + delta) : OOB);
        }
        return;
      }
      const uint32_t kofs = MN ? (uint32_t)(kt * BBK) * (uint32_t)p.lda * 2u : (uint32_t)(kt * BBK * 2);
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
        glds16(ra, base + (w * 64 + hh * BGT) * 8,
               kt * BBK + ka[hh] < klen ? va[h][hh] + kofs : OOB);
    } else {
      const uint32_t kofs = MNB ? (uint32_t)(kt * BBK) * (uint32_t)p.ldb * 2u : (uint32_t)(kt * BBK * 2);
      uint16_t* base = lds + buf * BUF + 2 * AHALF + (h - 2) * BHALF;
      if constexpr (GB) {
        // the chunk's output pixel (row kt*64 + kb of the K-slice) -> its window origin
#pragma unroll
        for (int hb = 0; hb < NB; ++hb) {
          const int kk = kt * BBK + kb[hb];
          const int pix = kbeg + (kk < klen ? kk : 0);
          int rem, x;
          const int b = fdivmod(pix, gHw, inv_hw, rem);
          const int y = fdivmod(rem, p.cv.cls[0].Wg, inv_wg, x);
          const int yb = y * p.cv.sh, xb = x * p.cv.sw;
          const bool ok = kk < klen && (unsigned)(yb + bho[h - 2][hb]) < (unsigned)gHin &&
                          (unsigned)(xb + bwo[h - 2][hb]) < (unsigned)gWin;
          const int pbase = ((b * gHin + yb) * gWin + xb) * gC * 2;
          glds16(rb, base + (w * 64 + hb * BGT) * 8, ok ? (uint32_t)(pbase + (int)vb[h - 2][hb]) : OOB);
        }
        return;
      }
#pragma unroll
      for (int hb = 0; hb < NB; ++hb)
        glds16(rb, base + (w * 64 + hb * BGT) * 8,
               kt * BBK + kb[hb] < klen ? vb[h - 2][hb] + kofs : OOB);
    }
  };

  f32x4 acc[2][2][4][FQ];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < FQ; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  h16x8 fa0[4][2], fa1[4][2], fb0[FQ][2], fb1[FQ][2];
  auto read_a = [&](h16x8 (&f)[4][2], const uint16_t* h) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if constexpr (MN) f[i][s] = frag_tr<128>(h, wm * 64 + i * 16, s);
        else f[i][s] = *reinterpret_cast<const h16x8*>(
            h + big_off(wm * 64 + i * 16 + (l & 15), 4 * s + (l >> 4)));
      }
  };
  auto read_b = [&](h16x8 (&f)[FQ][2], const uint16_t* h) {
#pragma unroll
    for (int j = 0; j < FQ; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if constexpr (MNB) f[j][s] = frag_tr<WB>(h, wn * QN + j * 16, s);
        else f[j][s] = *reinterpret_cast<const h16x8*>(
            h + big_off(wn * QN + j * 16 + (l & 15), 4 * s + (l >> 4)));
      }
  };
  auto mfma_q = [&](f32x4 (&c)[4][FQ], const h16x8 (&fa)[4][2], const h16x8 (&fb)[FQ][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < FQ; ++j)
          c[i][j] = mfma16(fb[j][s], fa[i][s], c[i][j]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto lgkm0 = [] { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
  auto bar = [] { __builtin_amdgcn_s_barrier(); };

  // prologue, in the steady-state issue order: (0,A0) (0,B0) (0,B1) (0,A1) (1,A0) (1,B0) (1,B1);
  // the wait retires the first two (the 5 half-tiles issued after them stay in flight)
  dma(0, 0, 0); dma(0, 0, 2); dma(0, 0, 3); dma(0, 0, 1);
  dma(1, 1, 0); dma(1, 1, 2); dma(1, 1, 3);
  vm_wait<VM_P3>();
  if (wm == 1) bar();                 // the stagger: wave row 1 runs one barrier behind row 0
  bar();
  for (int c = 0; c < T; ++c) {
    const int b = c & 1, nb = b ^ 1;
    const uint16_t* H = lds + b * BUF;
    // P0: Q00
    read_a(fa0, H);
    read_b(fb0, H + 2 * AHALF);
    dma(c + 1, nb, 1);                // (c+1).A1 -> buffer nb (its last reader: P2 of c-1)
    vm_wait<VM_P01>();                // retires (c).B1, read in P1
    lgkm0();
    bar();
    mfma_q(acc[0][0], fa0, fb0);
    bar();
    // P1: Q01
    read_b(fb1, H + 2 * AHALF + BHALF);
    dma(c + 2, b, 0);                 // (c+2).A0 -> buffer b (read in P0, retired before its barrier)
    vm_wait<VM_P01>();                // retires (c).A1, read in P2
    lgkm0();
    bar();
    mfma_q(acc[0][1], fa0, fb1);
    bar();
    // P2: Q11
    read_a(fa1, H + AHALF);
    dma(c + 2, b, 2);                 // (c+2).B0 (read in P0)
    lgkm0();
    bar();
    mfma_q(acc[1][1], fa1, fb1);
    bar();
    // P3: Q10 from registers
    dma(c + 2, b, 3);                 // (c+2).B1 (read in P1)
    vm_wait<VM_P3>();                 // retires (c+1).A0 and (c+1).B0, read in P0 of c+1
    bar();
    mfma_q(acc[1][0], fa1, fb0);
    bar();
  }
  // no LDS-DMA may land after the workgroup has released its LDS; row 0 takes the barrier row 1
  // took up front, so both rows have passed the same number when they leave
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (wm == 0) bar();

  // ---- epilogue, straight from the accumulators. B was the MFMA's first operand, so lane l holds
  // C[m = .. + (l & 15)][n = .. + 4 * (l >> 4) + r], r = 0..3.
  const bool vec4 = (EPI == EPI_PARTIAL ? (p.N & 3) == 0 : (p.ldc & 3) == 0);
  float* P = EPI == EPI_PARTIAL ? p.partial + (int64_t)split * p.M * p.N : nullptr;
  // EPI_STATS: Σv / Σv² of the stored (bf16-rounded) outputs per column over a wave row's 128
  // rows, folded across the 16 row-lanes in DPP rows; one statistics row per wave row (128 rows of
  // C: gemm.hip stats_rows_bm), written straight from the registers — no LDS, no barrier
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
#pragma unroll
    for (int j = 0; j < FQ; ++j) {
      const int nl = wn * (BN / 4) + qb * QN + j * 16 + 4 * (l >> 4);
      const int n = n0 + nl;
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if (EPI != EPI_PARTIAL && p.bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = n + r < p.N ? p.bias[n + r] : 0.f;
      }
      float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int qa = 0; qa < 2; ++qa)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = m0 + wm * 128 + qa * 64 + i * 16 + (l & 15);
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float x = acc[qa][qb][i][j][r];
            if (EPI != EPI_PARTIAL) {
              x += bv[r];
              if (p.relu) x = fmaxf(x, 0.f);
            }
            v[r] = x;
          }
          if (m >= p.M) continue;
          if (EPI == EPI_PARTIAL) {
            float* d = P + (int64_t)m * p.N + n;
            if (vec4 && n + 3 < p.N) *reinterpret_cast<float4*>(d) = make_float4(v[0], v[1], v[2], v[3]);
            else for (int r = 0; r < 4 && n + r < p.N; ++r) d[r] = v[r];
          } else if (p.out_bf16) {
            uint16_t h[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              h[r] = f2h(v[r]);
              v[r] = h2f(h[r]);
            }
            uint16_t* d = static_cast<uint16_t*>(p.C) + (int64_t)m * p.ldc + n;
            if (vec4 && n + 3 < p.N) {
              *reinterpret_cast<uint2*>(d) =
                  make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16));
            } else {
              for (int r = 0; r < 4 && n + r < p.N; ++r) d[r] = h[r];
            }
          } else {
            float* d = static_cast<float*>(p.C) + (int64_t)m * p.ldc + n;
            if (vec4 && n + 3 < p.N) {
              float4 o = make_float4(v[0], v[1], v[2], v[3]);
              if (p.accumulate) {
                const float4 q = *reinterpret_cast<const float4*>(d);
                o.x += q.x; o.y += q.y; o.z += q.z; o.w += q.w;
              }
              *reinterpret_cast<float4*>(d) = o;
            } else {
              for (int r = 0; r < 4 && n + r < p.N; ++r) d[r] = p.accumulate ? d[r] + v[r] : v[r];
            }
          }
          if (EPI == EPI_STATS) {
#pragma unroll
            for (int r = 0; r < 4; ++r) { s1[r] += v[r]; s2[r] += v[r] * v[r]; }
          }
        }
      if (EPI == EPI_STATS) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {      // the 16 row-lanes: one DPP row (gemm_core.h sum16)
          s1[r] = sum16(s1[r]);
          s2[r] = sum16(s2[r]);
        }
        const int srow = tm * 2 + wm;
        if ((l & 15) == 0 && srow * 128 < p.M && n < p.N) {
          float* d = p.stats + (int64_t)srow * 2 * p.N + n;
          *reinterpret_cast<float4*>(d) = make_float4(s1[0], s1[1], s1[2], s1[3]);
          *reinterpret_cast<float4*>(d + p.N) = make_float4(s2[0], s2[1], s2[2], s2[3]);
        }
      }
    }
}


// ---------------------------------------------------------------------------------------------
// Persistent form (GEMM_P256 / GEMM_P256x128) for K-contiguous A and B with a bf16 output: one
// workgroup per CU walks tiles blockIdx.x, +gridDim.x, ... and the K-tile schedule above runs on
// over the tile boundary: the last two K-tiles of tile j issue the DMAs of K-tiles 0 and 1 of tile
// j+1, so tile j's epilogue (stores straight from the accumulators, the statistics rows, the
// masked addend) overlaps the next tile's loads instead of every tile paying a cold pipeline fill
// and a workgroup launch. This is what the short-K, wide-N 1x1 convolutions of a ResNet need
// (K = 64..512 is 1-8 K-tiles: the fill and the epilogue were most of a tile's time).
// The epilogue ends with s_waitcnt vmcnt(0) (its stores and loads are then older than every later
// counted wait), so the counted waits of the next tile stay exact. The statistics rows are one per
// wave row, as in k_gemm_big. ADD: C = round(acc) + addend·[bit] (the residual gradient of a
// bottleneck's dx, gemm_core.h masked_addend), ldc == N.
template <int BN, bool STATS, bool ADD>
__global__ __launch_bounds__(BGT) void k_gemm_bigp(const GemmK p) {
  constexpr int BHALF = (BN / 2) * BBK;
  constexpr int BUF = 2 * AHALF + 2 * BHALF;
  constexpr int NB = BN / 128;
  constexpr int QN = BN / 8;
  constexpr int FQ = QN / 16;
  constexpr int VM_P01 = 3 * 2 + 2 * NB, VM_P3 = 2 * 2 + 3 * NB;
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * BUF];
  const int tiles_n = (p.N + BN - 1) / BN, tiles_m = (p.M + BBM - 1) / BBM;
  const int total = tiles_m * tiles_n;
  const int T = (p.K + BBK - 1) / BBK;             // >= 2 (host)
  const int klen = p.K;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
  const int wm = w >> 2, wn = w & 3;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, p.a_bytes), rb = make_rsrc(p.B, p.b_bytes);
  int ka[2], kb[NB];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const int q = threadIdx.x + hh * BGT;
    ka[hh] = ((q & 7) ^ ((q >> 3) & 7)) * 8;
  }
#pragma unroll
  for (int hb = 0; hb < NB; ++hb) {
    const int q = threadIdx.x + hb * BGT;
    kb[hb] = ((q & 7) ^ ((q >> 3) & 7)) * 8;
  }
  // DMA sources of a tile (see k_gemm_big): [0] the tile being computed, [1] the next one
  auto setup = [&](int t, uint32_t (&va)[2][2], uint32_t (&vb)[2][NB], int& m0, int& n0) {
    int tm, tn;
    tile_of(xcd_remap(t, total), tiles_m, tiles_n, tm, tn);
    m0 = tm * BBM;
    n0 = tn * BN;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int q = threadIdx.x + hh * BGT, lr = q >> 3;
#pragma unroll
      for (int qa = 0; qa < 2; ++qa) {
        const int row = m0 + (lr >> 6) * 128 + qa * 64 + (lr & 63);
        va[qa][hh] = row < p.M ? (uint32_t)(((int64_t)row * p.lda + ka[hh]) * 2) : OOB;
      }
    }
#pragma unroll
    for (int hb = 0; hb < NB; ++hb) {
      const int q = threadIdx.x + hb * BGT, lr = q >> 3;
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        const int col = n0 + (lr / QN) * (BN / 4) + qb * QN + (lr % QN);
        vb[qb][hb] = col < p.N ? (uint32_t)(((int64_t)col * p.ldb + kb[hb]) * 2) : OOB;
      }
    }
  };
  int t = blockIdx.x;
  uint32_t va[2][2], vb[2][NB], van[2][2], vbn[2][NB];
  int m0, n0, m0n = 0, n0n = 0;
  setup(t, va, vb, m0, n0);
  bool has_next = t + (int)gridDim.x < total;
  if (has_next) setup(t + gridDim.x, van, vbn, m0n, n0n);
  // K-tile kt of the current tile (kt >= T: K-tile kt - T of the next tile, or a zero-filling
  // OOB DMA past the last tile: the same number of DMA instructions in every phase)
  auto dma = [&](int kt, int buf, int h) {
    const bool nx = kt >= T;
    const int k = nx ? kt - T : kt;
    const bool live = !nx || has_next;
    if (h < 2) {
      uint16_t* base = lds + buf * BUF + h * AHALF;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const uint32_t v = nx ? van[h][hh] : va[h][hh];
        const bool ok = live && v != OOB && k * BBK + ka[hh] < klen;
        glds16(ra, base + (w * 64 + hh * BGT) * 8, ok ? v + (uint32_t)(k * BBK * 2) : OOB);
      }
    } else {
      uint16_t* base = lds + buf * BUF + 2 * AHALF + (h - 2) * BHALF;
#pragma unroll
      for (int hb = 0; hb < NB; ++hb) {
        const uint32_t v = nx ? vbn[h - 2][hb] : vb[h - 2][hb];
        const bool ok = live && v != OOB && k * BBK + kb[hb] < klen;
        glds16(rb, base + (w * 64 + hb * BGT) * 8, ok ? v + (uint32_t)(k * BBK * 2) : OOB);
      }
    }
  };
  f32x4 acc[2][2][4][FQ];
  h16x8 fa0[4][2], fa1[4][2], fb0[FQ][2], fb1[FQ][2];
  auto read_a = [&](h16x8 (&f)[4][2], const uint16_t* h) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        f[i][s] = *reinterpret_cast<const h16x8*>(h + big_off(wm * 64 + i * 16 + (l & 15), 4 * s + (l >> 4)));
  };
  auto read_b = [&](h16x8 (&f)[FQ][2], const uint16_t* h) {
#pragma unroll
    for (int j = 0; j < FQ; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        f[j][s] = *reinterpret_cast<const h16x8*>(h + big_off(wn * QN + j * 16 + (l & 15), 4 * s + (l >> 4)));
  };
  auto mfma_q = [&](f32x4 (&c)[4][FQ], const h16x8 (&fa)[4][2], const h16x8 (&fb)[FQ][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < FQ; ++j)
          c[i][j] = mfma16(fb[j][s], fa[i][s], c[i][j]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto lgkm0 = [] { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
  auto bar = [] { __builtin_amdgcn_s_barrier(); };

  dma(0, 0, 0); dma(0, 0, 2); dma(0, 0, 3); dma(0, 0, 1);
  dma(1, 1, 0); dma(1, 1, 2); dma(1, 1, 3);
  vm_wait<VM_P3>();
  if (wm == 1) bar();
  bar();
  int gb = 0;                          // buffer parity of this tile's K-tile 0
  for (;;) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < FQ; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < T; ++c) {
      const int b = (gb + c) & 1, nb = b ^ 1;
      const uint16_t* H = lds + b * BUF;
      read_a(fa0, H);
      read_b(fb0, H + 2 * AHALF);
      dma(c + 1, nb, 1);
      vm_wait<VM_P01>();
      lgkm0();
      bar();
      mfma_q(acc[0][0], fa0, fb0);
      bar();
      read_b(fb1, H + 2 * AHALF + BHALF);
      dma(c + 2, b, 0);
      vm_wait<VM_P01>();
      lgkm0();
      bar();
      mfma_q(acc[0][1], fa0, fb1);
      bar();
      read_a(fa1, H + AHALF);
      dma(c + 2, b, 2);
      lgkm0();
      bar();
      mfma_q(acc[1][1], fa1, fb1);
      bar();
      dma(c + 2, b, 3);
      vm_wait<VM_P3>();
      bar();
      mfma_q(acc[1][0], fa1, fb0);
      bar();
    }
    // ---- epilogue of this tile (the next tile's K-tiles 0 and 1 are in flight)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int j = 0; j < FQ; ++j) {
        const int n = n0 + wn * (BN / 4) + qb * QN + j * 16 + 4 * (l >> 4);
        float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int qa = 0; qa < 2; ++qa)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int m = m0 + wm * 128 + qa * 64 + i * 16 + (l & 15);
            const bool ok = m < p.M && n < p.N;
            const int64_t e = (int64_t)m * p.ldc + n;
            uint16_t h[4];
            float v[4];
            if constexpr (ADD) {
              // addend·[bit] added after rounding, as gemm_core.h add_h16x8 (one more rounding)
              uint2 ad = make_uint2(0u, 0u);
              uint32_t bits = 0xfu;
              if (ok) {
                ad = *reinterpret_cast<const uint2*>(p.addend + e);
                if (p.add_bits) bits = (uint32_t)(p.add_bits[e >> 3] >> (e & 7)) & 0xfu;
              }
              const uint32_t aw[2] = {ad.x, ad.y};
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float c0 = h_round(acc[qa][qb][i][j][r]);
                const uint32_t word = aw[r >> 1];
                const float av = ((bits >> r) & 1u) ? (r & 1 ? hhi(word) : hlo(word)) : 0.f;
                h[r] = f2h(c0 + av);
                v[r] = h2f(h[r]);
              }
            } else {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                h[r] = f2h(acc[qa][qb][i][j][r]);
                v[r] = h2f(h[r]);
              }
            }
            if (ok) {
              *reinterpret_cast<uint2*>(static_cast<uint16_t*>(p.C) + e) =
                  make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16));
            }
            if (STATS && ok) {
#pragma unroll
              for (int r = 0; r < 4; ++r) { s1[r] += v[r]; s2[r] += v[r] * v[r]; }
            }
          }
        if constexpr (STATS) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            s1[r] = sum16(s1[r]);
            s2[r] = sum16(s2[r]);
          }
          const int srow = (m0 / 128) + wm;
          if ((l & 15) == 0 && srow * 128 < p.M && n < p.N) {
            float* d = p.stats + (int64_t)srow * 2 * p.N + n;
            *reinterpret_cast<float4*>(d) = make_float4(s1[0], s1[1], s1[2], s1[3]);
            *reinterpret_cast<float4*>(d + p.N) = make_float4(s2[0], s2[1], s2[2], s2[3]);
          }
        }
      }
    // every epilogue access is now older than the next counted wait
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!has_next) break;
    gb = (gb + T) & 1;
    t += gridDim.x;
    m0 = m0n; n0 = n0n;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) va[a][hh] = van[a][hh];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int hb = 0; hb < NB; ++hb) vb[a][hb] = vbn[a][hb];
    has_next = t + (int)gridDim.x < total;
    if (has_next) setup(t + gridDim.x, van, vbn, m0n, n0n);
  }
  if (wm == 0) bar();
}

bool gemm_big_ok(const GemmArgs& g) {
  if (g.pro_scale != nullptr || g.addend != nullptr || g.bst_x != nullptr) return false;
  if (g.stats != nullptr && (g.N % 4) != 0) return false;      // float4 statistics rows
  if (g.a_kcontig && g.b_kcontig) return (g.K % 8) == 0 && (g.lda % 8) == 0 && (g.ldb % 8) == 0;
  if (g.a_kcontig && !g.b_kcontig)       // data gradient dY·W, W as stored ([K][N])
    return (g.K % 8) == 0 && (g.lda % 8) == 0 && (g.N % 8) == 0 && (g.ldb % 8) == 0;
  // both MN-contiguous: whole 16-byte column chunks
  return !g.a_kcontig && !g.b_kcontig && (g.M % 8) == 0 && (g.N % 8) == 0 && (g.lda % 8) == 0 &&
         (g.ldb % 8) == 0 && g.stats == nullptr;
}

// The big tiles for a row-gather convolution (conv.hip CV_A): one class with the identity row map,
// whole 64-channel K-tiles, a K-contiguous weight operand, no prologue / addend / backward
// statistics.
bool conv_big_ok(const GemmArgs& g, const ConvGeomHost& h) {
  if (!g.a_kcontig && !g.b_kcontig)          // weight gradient: B = the im2col column gather
    return h.nclass == 1 && h.C % 8 == 0 && g.M % 8 == 0 && g.N % 8 == 0 && (g.lda % 8) == 0 &&
           g.pro_scale == nullptr && g.stats == nullptr && !g.out_bf16;
  return h.nclass == 1 && h.osy == 1 && h.osx == 1 && h.C % BBK == 0 && g.b_kcontig &&
         (g.ldb % 8) == 0 && g.pro_scale == nullptr && g.addend == nullptr && g.bst_x == nullptr &&
         g.N % 8 == 0;
}

void conv_big(const GemmArgs& g, const GemmK& k, int zs, hipStream_t st) {
  const int bn = g.tile == GEMM_B256 ? 256 : 128;
  const int tiles = ((g.M + BBM - 1) / BBM) * ((g.N + bn - 1) / bn);
  const dim3 grid(tiles, zs), block(BGT);
  if (!g.a_kcontig) {                        // weight gradient (fp32 slab or accumulate)
#define LW_CBIGW(BNV)                                                                              \
  if (zs > 1) hipLaunchKernelGGL((k_gemm_big<BNV, EPI_PARTIAL, true, false, true>), grid, block, 0, st, k); \
  else hipLaunchKernelGGL((k_gemm_big<BNV, EPI_STORE, true, false, true>), grid, block, 0, st, k);
    if (bn == 256) { LW_CBIGW(256) } else { LW_CBIGW(128) }
#undef LW_CBIGW
    return;
  }
#define LW_CBIG(BNV)                                                                                \
  if (g.stats) hipLaunchKernelGGL((k_gemm_big<BNV, EPI_STATS, false, true>), grid, block, 0, st, k); \
  else hipLaunchKernelGGL((k_gemm_big<BNV, EPI_STORE, false, true>), grid, block, 0, st, k);
  if (bn == 256) { LW_CBIG(256) } else { LW_CBIG(128) }
#undef LW_CBIG
}

void gemm_big(const GemmArgs& g, const GemmK& k, int zs, hipStream_t st) {
  const int bn = g.tile == GEMM_B256 ? 256 : 128;
  const int tiles = ((g.M + BBM - 1) / BBM) * ((g.N + bn - 1) / bn);
  const dim3 grid(tiles, zs), block(BGT);
#define LW_BIG(BNV, MNV)                                                                         \
  if (zs > 1) hipLaunchKernelGGL((k_gemm_big<BNV, EPI_PARTIAL, MNV>), grid, block, 0, st, k);    \
  else if (g.stats) hipLaunchKernelGGL((k_gemm_big<BNV, EPI_STATS, MNV>), grid, block, 0, st, k); \
  else hipLaunchKernelGGL((k_gemm_big<BNV, EPI_STORE, MNV>), grid, block, 0, st, k);
  if (g.a_kcontig && !g.b_kcontig) {
#define LW_BIGX(BNV)                                                                                          \
  if (zs > 1) hipLaunchKernelGGL((k_gemm_big<BNV, EPI_PARTIAL, false, false, false, true>), grid, block, 0, st, k); \
  else if (g.stats) hipLaunchKernelGGL((k_gemm_big<BNV, EPI_STATS, false, false, false, true>), grid, block, 0, st, k); \
  else hipLaunchKernelGGL((k_gemm_big<BNV, EPI_STORE, false, false, false, true>), grid, block, 0, st, k);
    if (bn == 256) { LW_BIGX(256) } else { LW_BIGX(128) }
#undef LW_BIGX
  } else if (g.a_kcontig) {
    if (bn == 256) { LW_BIG(256, false) } else { LW_BIG(128, false) }
  } else {
    if (bn == 256) { LW_BIG(256, true) } else { LW_BIG(128, true) }
  }
#undef LW_BIG
}

// the persistent big tiles: K-contiguous operands, bf16 output without bias / ReLU / accumulate,
// no prologue / split-K / backward statistics, at least two K-tiles
bool gemm_bigp_ok(const GemmArgs& g) {
  if (!(g.a_kcontig && g.b_kcontig && g.out_bf16 && !g.accumulate && g.bias == nullptr &&
        !g.relu && g.pro_scale == nullptr && g.bst_x == nullptr && g.K > BBK))
    return false;
  if ((g.K % 8) != 0 || (g.lda % 8) != 0 || (g.ldb % 8) != 0 || (g.N % 8) != 0 || (g.ldc % 4) != 0)
    return false;
  if (g.add_bits != nullptr && g.ldc != g.N) return false;
  return true;
}

int cu_count() {
  int dev = 0, n = 0;
  (void)hipGetDevice(&dev);
  static int cached[64] = {0};
  if (dev >= 0 && dev < 64 && cached[dev] > 0) return cached[dev];
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
    n = 256;
  if (dev >= 0 && dev < 64) cached[dev] = n;
  return n;
}

void gemm_bigp(const GemmArgs& g, const GemmK& k, hipStream_t st) {
  const int bn = g.tile == GEMM_P256 ? 256 : 128;
  const int tiles = ((g.M + BBM - 1) / BBM) * ((g.N + bn - 1) / bn);
  const int grid = tiles < cu_count() ? tiles : cu_count();     // one workgroup per CU (LDS)
  const bool add = g.addend != nullptr, stats = g.stats != nullptr;
#define LW_P(BNV)                                                                                  \
  if (stats && add) hipLaunchKernelGGL((k_gemm_bigp<BNV, true, true>), dim3(grid), dim3(BGT), 0, st, k);  \
  else if (stats) hipLaunchKernelGGL((k_gemm_bigp<BNV, true, false>), dim3(grid), dim3(BGT), 0, st, k);   \
  else if (add) hipLaunchKernelGGL((k_gemm_bigp<BNV, false, true>), dim3(grid), dim3(BGT), 0, st, k);     \
  else hipLaunchKernelGGL((k_gemm_bigp<BNV, false, false>), dim3(grid), dim3(BGT), 0, st, k);
  if (bn == 256) { LW_P(256) } else { LW_P(128) }
#undef LW_P
}

}  // namespace lw
