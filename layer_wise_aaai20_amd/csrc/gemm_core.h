// 16-bit MFMA GEMM core for gfx950 (bf16, or fp16 in the lwaaai16 build: elem16.h), shared by the
// plain GEMM (gemm.hip) and the implicit-GEMM convolutions (conv.hip): tile staging, MFMA main
// loop and the fused epilogues.
// See gemm.hip for the design notes.
#pragma once
#include "common.h"
#include "lw_kernels.h"
#include "elem16.h"

namespace lw {

typedef short i16x4 __attribute__((ext_vector_type(4)));

constexpr int GT = 256;
constexpr int PAD = 8;                   // bf16 elements of padding per LDS row
enum { EPI_STORE = 0, EPI_PARTIAL = 1, EPI_STATS = 2, EPI_BSTATS = 3 };
enum { PRO_NONE = 0, PRO_A = 1, PRO_B = 2 };

// Sum over the 16 lanes of a DPP row, every lane getting the total: quad_perm [1,0,3,2] and
// [2,3,0,1] (partners l^1, l^2), row_half_mirror (partner 7-l: holds the other quad's identical
// sum, so equivalent to l^4) and row_mirror (15-l, equivalent to l^8). Each step is one VALU add
// with a DPP operand instead of a ds_bpermute round trip through the LDS crossbar, and the adds
// pair the same values in the same order as a l^1, l^2, l^4, l^8 butterfly (bit-identical).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                               0xF, 0xF, false));
}
__device__ __forceinline__ float sum16(float v) {
  v += dpp_mov<0xB1>(v);     // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);     // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);    // row_half_mirror
  v += dpp_mov<0x140>(v);    // row_mirror
  return v;
}

// 16-bit + 16-bit -> 16-bit per element (fp32 add, one rounding): the same arithmetic as a separate
// elementwise add of two bf16 tensors, so fusing the residual-gradient add changes no bits.
__device__ __forceinline__ uint4 add_h16x8(uint4 a, uint4 b) {
  const uint32_t x[4] = {a.x, a.y, a.z, a.w}, y[4] = {b.x, b.y, b.z, b.w};
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float lo = hlo(x[k]) + hlo(y[k]);
    const float hi = hhi(x[k]) + hhi(y[k]);
    w[k] = (uint32_t)f2h(lo) | ((uint32_t)f2h(hi) << 16);
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
  return h2f(add[e]);
}

// R = extent of the tile along m (A) or n (B). K-contiguous (KC) tiles are stored [R][BK]: at
// BK = 64 unpadded with the 16-byte chunks of row r XOR-swizzled (conflict-free ds_read_b128
// fragment reads, cdna_hip_programming.md T2), at BK = 32 padded to BK + 8. The M/N-contiguous
// tiles are stored [BK][R+PAD] and read with the transposing ds_read_b64_tr_b16. Both are moved as
// 16-byte chunks of 8 contiguous elements.
//
// MF is the MFMA shape the tile feeds: 16 (v_mfma_f32_16x16x32: a fragment read is 16 rows x one
// 8-k chunk per 16-lane group) or 32 (v_mfma_f32_32x32x16: 32 rows x one chunk per 32-lane half).
// The swizzle key differs: a ds_read_b128 is served in the lane groups {0-3,12-15,20-27},
// {4-11,16-19,28-31} (+32), so the 16 rows one group reads must hit 16 distinct 16-byte slots of
// the 256-byte bank row. Two 128-byte rows share a bank row (slot = 8*(r&1) + chunk'): for the
// 16x16 read (rows r&15 at chunks c, c+1) the key r & 7 does it; for the 32x32 read (rows
// {0-3,12-15,20-27} at ONE chunk) the key (r >> 1) & 7 does (r & 7 would leave it 2-way).
template <int MF>
__host__ __device__ constexpr int swz_key(int r) { return MF == 32 ? ((r >> 1) & 7) : (r & 7); }

template <int R, int BK, bool KC> struct Tile {
  static constexpr bool SWZ = KC && BK == 64;
  static constexpr int LD = KC ? (SWZ ? BK : BK + PAD) : R + PAD;
  static constexpr int ELEMS = KC ? R * LD : BK * LD;
  static constexpr int CPR = KC ? BK / 8 : R / 8;     // chunks per stored row
  static constexpr int PER_T = R * BK / 8 / GT;       // chunks per thread
  static_assert(R * BK / 8 % GT == 0, "tile must split evenly over the workgroup");
};

// M/N-contiguous tiles read by the 16x16x32 transposing fragment read (load_frag, MF = 16) are
// stored unpadded, R elements per row, with the 16-byte chunk c of row r at c ^ mn_swz<R>(r):
// a 32-lane half reads rows {8n .. 8n+3} of two 8-row groups at chunks 2j, 2j+1, and with the
// padded R + 8 layout those rows' 8-byte pieces overlapped in the 64 banks two by two (the weight
// gradients spent 42 % extra LDS cycles on conflicts: profiles/r6/pmc_conv3/). The swizzles make
// the 32 pieces land in 32 distinct bank pairs (R = 128: 256-byte rows, cdna_hip_programming.md
// T10 image (b); R = 64 / 256: the 128- / 512-byte-row forms checked the same way), and the
// register-staged chunk stores stay conflict-free (8 lanes, 8 consecutive chunks of one row).
// The 32x32x16 reads (MF = 32) keep the padded layout.
template <int R>
__host__ __device__ constexpr int mn_swz(int r) {
  return R == 128 ? (((r & 3) << 2) | ((r >> 2) & 3))
       : R == 64 ? ((((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2))
       : (((r & 3) << 1) | (r & 8));
}
template <int R, bool KC, int MF>
__host__ __device__ constexpr bool mn_swizzled() {
  return !KC && MF == 16 && (R == 64 || R == 128 || R == 256);
}

// element offset of chunk c of stored row r
template <int R, int BK, bool KC, int MF = 16>
__device__ __forceinline__ int tile_off(int r, int c) {
  using T = Tile<R, BK, KC>;
  if constexpr (mn_swizzled<R, KC, MF>()) return r * R + (c ^ mn_swz<R>(r & 15)) * 8;
  return r * T::LD + (T::SWZ ? (c ^ swz_key<MF>(r)) : c) * 8;
}

// Chunk i of the workgroup (thread t stages chunks t + h*GT): stored row rr, chunk column cc.
// GT is a multiple of CPR, so a thread's chunks all share one column.
template <int R, int BK, bool KC>
__device__ __forceinline__ void chunk_pos(int c, int& rr, int& cc) {
  using T = Tile<R, BK, KC>;
  rr = c / T::CPR;
  cc = c % T::CPR;
}

// ---- global loads: raw buffer loads. A chunk that must read as zero (outside the matrix, the K
// tail, the convolution padding) gets an offset past the buffer's end, and the hardware's range
// check returns zeros: no branches, no selects on the data.
constexpr uint32_t OOB = 0x80000000u;      // every operand is < 2 GiB (checked on the host)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ uint4 bload16(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0));
}
__device__ __forceinline__ uint2 bload8(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  return __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(r, voff, 0, 0));
}

// LDS-DMA staging (buffer_load_dwordx4 ... lds): 16 bytes per lane straight from memory into LDS
// at the wave-uniform base `wave_dst` + 16 * lane, no VGPRs and no ds_write. A range-checked
// (OOB) source writes zeros (scripts/probes/glds_oob_probe.hip, run on MI355X), so the
// convolution padding / matrix edges work exactly as with the register loads.
#ifndef LW_GLDS
#define LW_GLDS 1
#endif
__device__ __forceinline__ void glds16(__amdgpu_buffer_rsrc_t r, uint16_t* wave_dst, uint32_t voff) {
  typedef __attribute__((address_space(3))) void* lds_ptr;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr)wave_dst, 16, voff, 0, 0, 0);
}

// A K-contiguous BK = 64 tile filled by LDS-DMA: every wave-instruction writes 1 KiB = 8 whole
// 128-byte rows in lane order, so the XOR swizzle moves to the SOURCE: the lane that lands in
// stored chunk slot cc of row rr fetches logical chunk cc ^ key(rr). A thread's rows all share
// the key (they differ by multiples of GT / 8 = 32 rows), so one per-thread chunk column serves all.
template <int R, int BK, bool KC, bool DMA, int MF = 16>
__device__ __forceinline__ int src_chunk(int cc, int rr) {
  return (DMA && Tile<R, BK, KC>::SWZ) ? (cc ^ swz_key<MF>(rr)) : cc;
}

// LDS element offset of the first row of wave-instruction h of this thread's wave
template <int R, int BK, bool KC>
__device__ __forceinline__ int dma_wave_off(int h) {
  using T = Tile<R, BK, KC>;
  return (((int)(threadIdx.x & ~63u) + h * GT) / T::CPR) * T::LD;
}

// Plain operand tile: byte offset of each of this thread's chunks at k = 0 (OOB outside the
// matrix); a K-step adds k*2 (KC) or k*ld*2 (M/N-contiguous) and masks the K tail.
template <int R, int BK, bool KC, int MF = 16>
struct PlainLoader {
  static constexpr int PT = Tile<R, BK, KC>::PER_T;
  __amdgpu_buffer_rsrc_t rs;
  uint32_t voff[PT];
  int kpos[PT];       // k of each chunk within the step (KC: the chunk column, else its row)
  uint32_t ld2;

  template <bool DMA = false>
  __device__ __forceinline__ void init(const uint16_t* P, uint32_t bytes, int64_t ld, int row0,
                                       int rows) {
    rs = make_rsrc(P, bytes);
    ld2 = (uint32_t)(ld * 2);
#pragma unroll
    for (int h = 0; h < PT; ++h) {
      int rr, cc;
      chunk_pos<R, BK, KC>(threadIdx.x + h * GT, rr, cc);
      cc = src_chunk<R, BK, KC, DMA, MF>(cc, rr);
      if (KC) {
        const int gr = row0 + rr;
        voff[h] = gr < rows ? (uint32_t)(((int64_t)gr * ld + cc * 8) * 2) : OOB;
        kpos[h] = cc * 8;
      } else {
        const int gc = row0 + cc * 8;
        voff[h] = gc < rows ? (uint32_t)((int64_t)rr * ld * 2 + gc * 2) : OOB;
        kpos[h] = rr;
      }
    }
  }

  __device__ __forceinline__ void load(uint4 (&r)[PT], uint32_t (&okmask), int k, int kend) const {
    const uint32_t kb = KC ? (uint32_t)k * 2u : (uint32_t)k * ld2;
    okmask = 0;
#pragma unroll
    for (int h = 0; h < PT; ++h) {
      const bool ok = voff[h] != OOB && k + kpos[h] < kend;
      r[h] = bload16(rs, ok ? voff[h] + kb : OOB);
      okmask |= (ok ? 1u : 0u) << h;
    }
  }

  // the same chunks by LDS-DMA into tile S (init<true>)
  __device__ __forceinline__ void dma(uint16_t* S, int k, int kend) const {
    const uint32_t kb = KC ? (uint32_t)k * 2u : (uint32_t)k * ld2;
#pragma unroll
    for (int h = 0; h < PT; ++h) {
      const bool ok = voff[h] != OOB && k + kpos[h] < kend;
      glds16(rs, S + dma_wave_off<R, BK, KC>(h), ok ? voff[h] + kb : OOB);
    }
  }
};

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
    const float lo = fmaxf(fmaf(hlo(w[k]), c.s[2 * k], c.t[2 * k]), 0.f);
    const float hi = fmaxf(fmaf(hhi(w[k]), c.s[2 * k + 1], c.t[2 * k + 1]), 0.f);
    w[k] = (uint32_t)f2h(lo) | ((uint32_t)f2h(hi) << 16);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

template <int R, int BK, bool KC, bool PRO, int MF = 16>
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
    *reinterpret_cast<uint4*>(S + tile_off<R, BK, KC, MF>(rr, cc)) = v;
  }
}

// MFMA operand fragment: 8 bf16 along k.
//   MF = 16: k-group g = lane>>4, sub-step s of 32 k, tile row/col i_base + (lane&15);
//   MF = 32: k-group h = lane>>5, sub-step s of 16 k, tile row/col i_base + (lane&31).
// The transposing read (M/N-contiguous tiles): per 16-lane group, lane 4q+p addresses row q of a
// 4-row block at columns 4p..4p+3 and receives column (lane&15) of those 4 rows (T10); two reads
// (rows +0..3, +4..7) make the 8 k of a fragment. For MF = 32 the group's 16 columns are
// i_base + 16(g&1) + (lane&15) and its rows start at 16s + 8(g>>1).
template <int R, int BK, bool KC, int MF = 16>
__device__ __forceinline__ h16x8 load_frag(const uint16_t* S, int i_base, int s) {
  using T = Tile<R, BK, KC>;
  const int l = threadIdx.x & 63;
  if (MF == 32) {
    if (KC) {
      const uint16_t* p = S + tile_off<R, BK, KC, MF>(i_base + (l & 31), 2 * s + (l >> 5));
      return *reinterpret_cast<const h16x8*>(p);
    }
    const int g = l >> 4, t = l & 15, q = t >> 2, p4 = t & 3;
    typedef __attribute__((address_space(3))) i16x4 lds_v4;
    const uint16_t* p0 = S + (16 * s + 8 * (g >> 1) + q) * T::LD + i_base + 16 * (g & 1) + 4 * p4;
    const uint16_t* p1 = p0 + 4 * T::LD;
    const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(p0));
    const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(p1));
    typedef short i16x8 __attribute__((ext_vector_type(8)));
    const i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(h16x8, v);
  }
  if (KC) {
    const uint16_t* p = S + tile_off<R, BK, KC>(i_base + (l & 15), 4 * s + (l >> 4));
    return *reinterpret_cast<const h16x8*>(p);
  } else {
    const int g = l >> 4, t = l & 15, q = t >> 2, p4 = t & 3;
    typedef __attribute__((address_space(3))) i16x4 lds_v4;
    const uint16_t* p0;
    const uint16_t* p1;
    if constexpr (mn_swizzled<R, KC, MF>()) {
      const int r0 = 32 * s + 8 * g + q, col = i_base + 4 * p4;
      p0 = S + tile_off<R, BK, KC, MF>(r0, col >> 3) + (col & 7);
      p1 = S + tile_off<R, BK, KC, MF>(r0 + 4, col >> 3) + (col & 7);
    } else {
      p0 = S + (32 * s + 8 * g + q) * T::LD + i_base + 4 * p4;
      p1 = p0 + 4 * T::LD;
    }
    const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(p0));
    const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(p1));
    typedef short i16x8 __attribute__((ext_vector_type(8)));
    const i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(h16x8, v);
  }
}

__device__ __forceinline__ void store_out8(void* C, int64_t off, const float v[8], bool bf) {
  if (bf) {
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = (uint32_t)f2h(v[2 * k]) | ((uint32_t)f2h(v[2 * k + 1]) << 16);
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
  uint32_t a_bytes, b_bytes;   // operand extents for the buffer loads' range check
  // EPI_BSTATS (lw_kernels.h GemmArgs): x of the BN whose backward reduction the epilogue does
  const uint16_t* bst_x;
  const float* bst_mean;
  const float* bst_scale;
  const float* bst_shift;
  const uint8_t* bst_bits;
};

// q = a / d, r = a % d for 0 <= a < 2^24 via the fp32 reciprocal (one correction step each way:
// the estimate is off by at most one) — the per-thread pixel decode of the B gather.
__device__ __forceinline__ int fdivmod(int a, int d, float inv, int& r) {
  int q = (int)((float)a * inv);
  r = a - q * d;
  if (r < 0) { --q; r += d; }
  else if (r >= d) { ++q; r -= d; }
  return q;
}

// ---- A-gather (im2col rows), K-contiguous tile. Per thread and chunk, fixed for the K loop:
// the byte offset of the chunk's pixel at tap (0, 0) and channel cc*8, and the pixel's window
// origin (hb, wb; rows past the class's M get an origin that fails every bounds test).
// Per K-step with C % BK == 0 the whole step lies in one tap: tap and first channel are uniform
// (scalar unit), and a chunk costs an add, two bounds tests and a select. Otherwise (C == 4, the
// image; or C < BK) every chunk decodes its own tap.
template <int R, int BK>
struct RowGather {
  static constexpr int PT = Tile<R, BK, true>::PER_T;
  __amdgpu_buffer_rsrc_t rs;
  int rowoff[PT];       // bytes; may be negative (window origin in the padding)
  int hb[PT], wb[PT];
  int kc;               // this thread's k offset within a step (cc*8)
  int ci0, js, jr;      // fast path: tap and first channel of the next K-step (uniform)
  int c4_drow, c4_js;   // 4-channel image: the thread's tap relative to the step's first row
};

template <int R, int BK, bool DMA = false, int MF = 16>
__device__ __forceinline__ void row_gather_init(RowGather<R, BK>& g, const uint16_t* X,
                                                uint32_t bytes, const ConvGeom& cv,
                                                const ConvClass& cc, int m0) {
  using T = Tile<R, BK, true>;
  g.rs = make_rsrc(X, bytes);
  const int hw = cc.Hg * cc.Wg;
  g.kc = src_chunk<R, BK, true, DMA, MF>((int)(threadIdx.x % T::CPR), (int)(threadIdx.x / T::CPR)) * 8;
  // 4-channel gather with BK a multiple of a whole filter row (4*TS elements): a K-step covers
  // whole rows, so the thread's tap offset within them is fixed (no per-chunk division)
  g.c4_drow = (g.kc >> 2) / cc.TS;
  g.c4_js = (g.kc >> 2) - g.c4_drow * cc.TS;
#pragma unroll
  for (int h = 0; h < T::PER_T; ++h) {
    int rr, c8;
    chunk_pos<R, BK, true>(threadIdx.x + h * GT, rr, c8);
    const int m = m0 + rr;
    const bool in = m < cc.M;
    const int mm = in ? m : 0;                   // (branch-free: see load_coef8)
    const int b = mm / hw, rem = mm - b * hw;
    const int y = rem / cc.Wg, x = rem - y * cc.Wg;
    const int h0 = y * cv.sh + cc.oh, w0 = x * cv.sw + cc.ow;
    g.hb[h] = in ? h0 : -(1 << 28);
    g.wb[h] = w0;
    g.rowoff[h] = (((b * cv.Hin + h0) * cv.Win + w0) * cv.C + g.kc) * 2;
  }
}

// fast path: position the uniform tap walk at K-step k (divisions once per kernel)
template <int R, int BK>
__device__ __forceinline__ void row_gather_seek(RowGather<R, BK>& g, const ConvGeom& cv,
                                                const ConvClass& cc, int k) {
  const int t = k / cv.C;
  g.ci0 = k - t * cv.C;
  g.jr = t / cc.TS;
  g.js = t - g.jr * cc.TS;
}

template <int R, int BK, bool C4, bool DMA = false>
__device__ __forceinline__ void load_tile_gather_a(const ConvGeom& cv, const ConvClass& cc,
                                                   RowGather<R, BK>& g, int k, int kend,
                                                   uint4 (&r)[Tile<R, BK, true>::PER_T],
                                                   int& ci_out, uint32_t& okmask,
                                                   uint16_t* S = nullptr) {
  using T = Tile<R, BK, true>;
  static_assert(!(DMA && C4), "4-channel gathers stage through registers");
  okmask = 0;
  const bool kin = k + g.kc < kend;
  if (!C4 && cv.C % BK == 0) {
    // the whole K-step lies in one tap: uniform tap / channel arithmetic, walked incrementally
    // (the K-steps are fetched in order; row_gather_seek positioned the walk at the first)
    const int ho = cv.dh * g.jr, wo = cv.dw * g.js;
    const int delta = ((ho * cv.Win + wo) * cv.C + g.ci0) * 2;
    ci_out = g.ci0 + g.kc;
    g.ci0 += BK;
    if (g.ci0 >= cv.C) {
      g.ci0 = 0;
      if (++g.js == cc.TS) { g.js = 0; ++g.jr; }
    }
#pragma unroll
    for (int h = 0; h < T::PER_T; ++h) {
      const bool ok = kin && (unsigned)(g.hb[h] + ho) < (unsigned)cv.Hin &&
                      (unsigned)(g.wb[h] + wo) < (unsigned)cv.Win;
      const uint32_t off = ok ? (uint32_t)(g.rowoff[h] + delta) : OOB;
      if constexpr (DMA) glds16(g.rs, S + dma_wave_off<R, BK, true>(h), off);
      else r[h] = bload16(g.rs, off);
      okmask |= (ok ? 1u : 0u) << h;
    }
    return;
  }
  // per-thread tap decode (the chunk's k is k + kc)
  const int kk = k + g.kc;
  int t, ci, jr, js;
  if (C4 && BK % (4 * cc.TS) == 0) {      // whole filter rows per step: uniform row, fixed tap
    ci = 0;
    jr = k / (4 * cc.TS) + g.c4_drow;
    js = g.c4_js;
  } else {
    if (C4) { t = kk >> 2; ci = 0; }
    else { t = kk / cv.C; ci = kk - t * cv.C; }
    jr = t / cc.TS;
    js = t - jr * cc.TS;
  }
  const int ho = cv.dh * jr, wo = cv.dw * js;
  // rowoff holds channel kc: rebase it on (tap, ci)
  const int delta = ((ho * cv.Win + wo) * cv.C + ci - g.kc) * 2;
  ci_out = ci;
#pragma unroll
  for (int h = 0; h < T::PER_T; ++h) {
    const int hi = g.hb[h] + ho, wi = g.wb[h] + wo;
    const bool row_ok = kin && (unsigned)hi < (unsigned)cv.Hin;
    const uint32_t off = (uint32_t)(g.rowoff[h] + delta);
    if (C4) {
      // pixels wi and wi + dw of a 4-channel (8-byte) image
      const bool ok0 = row_ok && (unsigned)wi < (unsigned)cv.Win;
      const bool ok1 = row_ok && (unsigned)(wi + cv.dw) < (unsigned)cv.Win;
      const uint2 a = bload8(g.rs, ok0 ? off : OOB);
      const uint2 b = bload8(g.rs, ok1 ? off + cv.dw * 8 : OOB);
      r[h] = make_uint4(a.x, a.y, b.x, b.y);
      okmask |= (ok0 || ok1 ? 1u : 0u) << h;
    } else {
      const bool ok = row_ok && (unsigned)wi < (unsigned)cv.Win;
      if constexpr (DMA) glds16(g.rs, S + dma_wave_off<R, BK, true>(h), ok ? off : OOB);
      else r[h] = bload16(g.rs, ok ? off : OOB);
      okmask |= (ok ? 1u : 0u) << h;
    }
  }
}

#ifndef LW_BGATHER_IL
#define LW_BGATHER_IL 1     // interleaved B-gather chunks (store_tile_rows); 0: runs of PER_T
#endif
// ---- B-gather (weight gradient): N-contiguous tile whose rows are output pixels and whose
// chunks are (tap, 8 channels) — or C4: (tap pair, 4 channels) — of the input. Here a thread
// stages PER_T chunks of ONE row (row-major chunk order instead of chunk_pos), so the pixel
// decode is done once per thread per K-step.
template <int R, int BK>
struct ColGather {
  static constexpr int PT = Tile<R, BK, false>::PER_T;
  static constexpr int TPR = Tile<R, BK, false>::CPR / PT;   // threads per stored row
  static_assert(Tile<R, BK, false>::CPR % PT == 0, "row-major B gather split");
  __amdgpu_buffer_rsrc_t rs;
  int tapoff[PT];       // bytes: (hoff*Win + woff)*C*2 + ci*2
  int hoff[PT], woff[PT];
  uint32_t nok;         // chunk h inside N
  int rr;               // this thread's row within the K-step
  int hw;
  float inv_hw, inv_w;
};

template <int R, int BK, bool C4>
__device__ __forceinline__ void col_gather_init(ColGather<R, BK>& g, const uint16_t* X,
                                                uint32_t bytes, const ConvGeom& cv,
                                                const ConvClass& cc, int n0, int N) {
  using G = ColGather<R, BK>;
  g.rs = make_rsrc(X, bytes);
  g.rr = threadIdx.x / G::TPR;
  g.hw = cc.Hg * cc.Wg;
  g.inv_hw = 1.f / (float)g.hw;
  g.inv_w = 1.f / (float)cc.Wg;
  g.nok = 0;
#pragma unroll
  for (int h = 0; h < G::PT; ++h) {
    const int nn = n0 + (LW_BGATHER_IL ? h * G::TPR + (int)(threadIdx.x % G::TPR)
                                       : (int)(threadIdx.x % G::TPR) * G::PT + h) * 8;
    int t, ci;
    if (C4) { t = nn >> 2; ci = 0; }
    else { t = nn / cv.C; ci = nn - t * cv.C; }
    const int jr = t / cc.TS, js = t - jr * cc.TS;
    g.hoff[h] = cc.oh + cv.dh * jr;
    g.woff[h] = cc.ow + cv.dw * js;
    g.tapoff[h] = ((g.hoff[h] * cv.Win + g.woff[h]) * cv.C + ci) * 2;
    g.nok |= (nn < N ? 1u : 0u) << h;
  }
}

template <int R, int BK, bool C4>
__device__ __forceinline__ void load_tile_gather_b(const ConvGeom& cv, const ColGather<R, BK>& g,
                                                   int k, int kend,
                                                   uint4 (&r)[Tile<R, BK, false>::PER_T],
                                                   uint32_t& okmask) {
  using G = ColGather<R, BK>;
  const int pix = k + g.rr;
  int rem, x;
  const int b = fdivmod(pix, g.hw, g.inv_hw, rem);
  const int y = fdivmod(rem, cv.cls[0].Wg, g.inv_w, x);
  const int yb = y * cv.sh, xb = x * cv.sw;
  const int base = ((b * cv.Hin + yb) * cv.Win + xb) * cv.C * 2;
  const bool pok = pix < kend;
  okmask = 0;
#pragma unroll
  for (int h = 0; h < G::PT; ++h) {
    const int hi = yb + g.hoff[h], wi = xb + g.woff[h];
    const bool row_ok = pok && ((g.nok >> h) & 1u) && (unsigned)hi < (unsigned)cv.Hin;
    const uint32_t off = (uint32_t)(base + g.tapoff[h]);
    if (C4) {
      const bool ok0 = row_ok && (unsigned)wi < (unsigned)cv.Win;
      const bool ok1 = row_ok && (unsigned)(wi + cv.dw) < (unsigned)cv.Win;
      const uint2 a = bload8(g.rs, ok0 ? off : OOB);
      const uint2 c = bload8(g.rs, ok1 ? off + cv.dw * 8 : OOB);
      r[h] = make_uint4(a.x, a.y, c.x, c.y);
      okmask |= (ok0 || ok1 ? 1u : 0u) << h;
    } else {
      const bool ok = row_ok && (unsigned)wi < (unsigned)cv.Win;
      r[h] = bload16(g.rs, ok ? off : OOB);
      okmask |= (ok ? 1u : 0u) << h;
    }
  }
}

// store of a B-gather tile (row-major chunk order, see ColGather). A row's TPR threads take its
// chunks interleaved (chunk h·TPR + t % TPR, not a run of PT per thread): with a run, the 8 lanes
// of a ds_write_b128 group stored chunks PT apart, i.e. into the same 16-byte bank slots (2- to
// 4-way conflicts); interleaved, they store 4-8 consecutive chunks of a row, and the tile's row
// swizzle puts the next row's chunks in the other slots.
template <int R, int BK, int MF = 16>
__device__ __forceinline__ void store_tile_rows(uint16_t* __restrict__ S,
                                                const uint4 (&r)[Tile<R, BK, false>::PER_T]) {
  using G = ColGather<R, BK>;
  const int rr = threadIdx.x / G::TPR, c0 = threadIdx.x % G::TPR;
#pragma unroll
  for (int h = 0; h < G::PT; ++h) {
    const int c = LW_BGATHER_IL ? h * G::TPR + c0 : c0 * G::PT + h;
    *reinterpret_cast<uint4*>(S + tile_off<R, BK, false, MF>(rr, c)) = r[h];
  }
}

// LDS-DMA ring depth: bytes in flight per CU, not K-steps, hide the L2/Infinity-Cache latency
// (Little's law: ~64 KB in flight caps a 128x128 tile at ~40 % of the MFMA rate). LW_NSTAGE
// overrides for experiments.
#ifndef LW_NSTAGE
#define LW_NSTAGE 2
#endif
__host__ __device__ constexpr int dma_stages(int bm, int bn) {
  return (bm + bn) * 64 * 2 * LW_NSTAGE <= 160 * 1024 - 8192 ? LW_NSTAGE : 2;
}

// Wait until at most `ahead` K-steps (PER DMAs each) of this wave are still in flight, then
// barrier. Inline asm with a memory clobber: a __syncthreads() would drain every DMA (vmcnt(0)).
template <int N>
__device__ __forceinline__ void vm_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}
template <int NS, int PER>
__device__ __forceinline__ void dma_wait_barrier(int ahead) {
  static_assert((NS - 2) * PER <= 63, "vmcnt is 6 bits");
  if (NS >= 4 && ahead >= 2) vm_wait_barrier<(NS >= 4 ? 2 * PER : 0)>();
  else if (NS >= 3 && ahead >= 1) vm_wait_barrier<(NS >= 3 ? PER : 0)>();
  else vm_wait_barrier<0>();
}

// Workgroup id → (m-tile, n-tile): consecutive ids are dealt round-robin to the 8 XCDs, so remap
// each XCD's share onto one contiguous range of the row-major tile order.
__device__ __forceinline__ int xcd_remap(int pid, int total) {
  const int q = total >> 3, rem = total & 7;
  const int x = pid & 7, idx = pid >> 3;
  return x * q + (x < rem ? x : rem) + idx;
}

// Tile order within an XCD's contiguous range: groups of GROUP_M tile rows, column-major inside
// a group, so the ~64 workgroups an XCD holds at once cover a GROUP_M x (64 / GROUP_M) block of
// tiles and share GROUP_M A row-panels and as many B column-panels in its L2 — instead of one A
// panel and 64 B panels (row-major). Skinny-M problems (tiles_m <= GROUP_M, e.g. a classifier at
// batch 512) become column-major: each XCD streams its own slice of the large weight operand.
constexpr int GROUP_M = 8;
__device__ __forceinline__ void tile_of(int pid, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int per_group = GROUP_M * tiles_n;
  const int g = pid / per_group, first = g * GROUP_M;
  const int rows = min(tiles_m - first, GROUP_M);
  const int r = pid - g * per_group;
  tm = first + r % rows;
  tn = r / rows;
}

#ifndef LW_SPLIT_XCD
#define LW_SPLIT_XCD 1           // 0: split = blockIdx.y, tiles remapped within a slice only (A/B)
#endif
// (tile, split-K slice) of this workgroup. Workgroups are dealt to the 8 XCDs round-robin in
// dispatch order (x fastest, then y); remap that order so each XCD gets one contiguous range of the
// split-major (slice, tile) order: the tiles of one K-slice then sit on the same XCD and share
// their common operand rows in its L2 (a weight gradient's im2col columns of one pixel range are
// read by every column tile) instead of each fetching them from HBM. zs == 1: the plain map.
__device__ __forceinline__ void tile_split_of(int tiles_m, int tiles_n, int& tm, int& tn,
                                              int& split) {
  const int tiles = tiles_m * tiles_n;
  if (gridDim.y == 1 || !LW_SPLIT_XCD) {
    split = (int)blockIdx.y;
    tile_of(xcd_remap(blockIdx.x, tiles), tiles_m, tiles_n, tm, tn);
    return;
  }
  const int lin = xcd_remap((int)(blockIdx.y * gridDim.x + blockIdx.x), tiles * (int)gridDim.y);
  split = lin / tiles;
  tile_of(lin - split * tiles, tiles_m, tiles_n, tm, tn);
}

template <int MF> struct AccOf { typedef f32x4 T; };
template <> struct AccOf<32> { typedef f32x16 T; };

// Sum over the 32 lanes of one half-wave, every lane getting the total: the 16-lane DPP fold,
// then the other DPP row of the half (ds_swizzle bit mode, xor 16): both lanes of a pair add the
// same two values, so every lane holds the bit-identical total.
__device__ __forceinline__ float sum32(float v) {
  v = sum16(v);
  return v + __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v),
                                                                    0x401F));
}

// MF: the MFMA shape (16: v_mfma_f32_16x16x32, 32: v_mfma_f32_32x32x16). Same tiles, waves and
// LDS traffic per FLOP (a wave's WTM x WTN block reads (WTM + WTN) x BK operands per K-step either
// way); the 32x32 shape issues half the MFMA instructions, its operand fragments cover 32 rows,
// and its accumulators hold four runs of 4 consecutive columns per lane.
template <int BM, int BN, int BK, bool AKC, bool BKC, int EPI, int PRO, int CV = CV_NONE,
          int MF = 16>
__global__ __launch_bounds__(GT) void k_gemm(const GemmK p) {
  using TA = Tile<BM, BK, AKC>;
  using TB = Tile<BN, BK, BKC>;
  using Acc = typename AccOf<MF>::T;
  constexpr int WTM = BM / 2, WTN = BN / 2, FM = WTM / MF, FN = WTN / MF;
  constexpr int NG = MF == 32 ? 4 : 1;         // runs of 4 consecutive columns per accumulator
  constexpr int NR = MF == 32 ? 16 : 4;        // accumulator registers
  static_assert(WTM % MF == 0 && WTN % MF == 0, "wave tile must hold whole MFMA blocks");
  constexpr int STAGE = TA::ELEMS + TB::ELEMS;
  constexpr int LDC = BN + 4;                  // fp32 staging row (≡ 4 dwords mod 64 banks)
  constexpr int LDH = BN + 16;                 // bf16 staging row (≡ 8 dwords mod 64 banks)
  constexpr int CS_BYTES = WTM * LDC * 4;
  constexpr int CH_BYTES = BM * LDH * 2 + 2 * 2 * BN * 4;
  // both operands K-contiguous BK = 64 swizzled tiles, no prologue: stage by LDS-DMA
  constexpr bool GL = LW_GLDS && AKC && BKC && BK == 64 && PRO == PRO_NONE &&
                      (CV == CV_NONE || CV == CV_A);
  constexpr int NS = GL ? dma_stages(BM, BN) : 2;    // LDS stages (ring)
  constexpr int ST_BYTES = NS * STAGE * 2;
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
  int tm, tn;
  int split;
  tile_split_of(tiles_m, tiles_n, tm, tn, split);
  const int m0 = tm * BM, n0 = tn * BN;
  // the class record by constant index (a runtime index into the by-value kernel argument
  // would copy the whole array to scratch)
  const int zc = GA ? (int)blockIdx.z : 0;
  const ConvClass ccl = zc == 0 ? p.cv.cls[0] : zc == 1 ? p.cv.cls[1]
                      : zc == 2 ? p.cv.cls[2] : p.cv.cls[3];
  if (GA && m0 >= ccl.M) return;                // parity class with fewer rows than the grid
  const int Kc = GA ? ccl.K : p.K;
  const int kbeg = split * p.k_per_split;
  const int kend = min(Kc, kbeg + p.k_per_split);
  const uint16_t* Bp = GA ? p.B + ccl.b_off : p.B;
  const int Mrow = GA ? ccl.M : p.M;             // valid GEMM rows of this workgroup
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int wr = w >> 1, wc = w & 1;

  Acc acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < NR; ++r) acc[i][j][r] = 0.f;

  // One register staging set: the next K-step's global loads are issued before this step's
  // MFMAs and written to the other LDS buffer after them. (A second set — loads two steps
  // ahead — measured no faster: the loop is bound by the L2→CU operand traffic of the tile,
  // not by load latency; profiles/r2_conv_fusion_variants.log.)
  struct Regs {
    uint4 a[TA::PER_T], b[TB::PER_T];
    uint32_t oka, okb;
    Coef8 coA;
  };
  Regs R0;
  Coef8 coB;
  RowGather<BM, BK> rg;
  ColGather<BN, BK> cg;
  PlainLoader<BM, BK, AKC, MF> la;
  PlainLoader<BN, BK, BKC, MF> lb;
  if constexpr (GA) {
    row_gather_init<BM, BK, GL, MF>(rg, p.A, p.a_bytes, p.cv, ccl, m0);
    if (!G4 && p.cv.C % BK == 0) row_gather_seek<BM, BK>(rg, p.cv, ccl, kbeg);
  } else {
    la.template init<GL>(p.A, p.a_bytes, p.lda, m0, p.M);
  }
  if constexpr (GB) col_gather_init<BN, BK, G4>(cg, p.B, p.b_bytes, p.cv, ccl, n0, p.N);
  else lb.template init<GL>(Bp, p.b_bytes - (uint32_t)((Bp - p.B) * 2), p.ldb, n0, p.N);
  static_assert(!GB || PRO != PRO_B, "B-gather prologue: materialise the input instead");
  if (PRO == PRO_B)        // channel n of this thread's B chunks: fixed for the whole kernel
    load_coef8(coB, p.pro_scale, p.pro_shift, n0 + (threadIdx.x % TB::CPR) * 8, p.N);
  const int a_koff = (threadIdx.x % TA::CPR) * 8;      // PRO_A: k offset within a K-step
  // global -> registers for the K-step at k (and, PRO_A, its prologue coefficients)
  auto fetch = [&](int k, Regs& r) {
    int a_ch = k + a_koff;
    if constexpr (GA) load_tile_gather_a<BM, BK, G4>(p.cv, ccl, rg, k, kend, r.a, a_ch, r.oka);
    else la.load(r.a, r.oka, k, kend);
    if constexpr (GB) load_tile_gather_b<BN, BK, G4>(p.cv, cg, k, kend, r.b, r.okb);
    else lb.load(r.b, r.okb, k, kend);
    if (PRO == PRO_A) load_coef8(r.coA, p.pro_scale, p.pro_shift, a_ch, GA ? p.cv.C : kend);
  };
  auto stage = [&](uint16_t* dst, const Regs& r) {
    store_tile<BM, BK, AKC, PRO == PRO_A, MF>(dst, r.a, r.oka, r.coA);
    if constexpr (GB) store_tile_rows<BN, BK, MF>(dst + TA::ELEMS, r.b);
    else store_tile<BN, BK, BKC, PRO == PRO_B, MF>(dst + TA::ELEMS, r.b, r.okb, coB);
  };
  auto compute = [&](const uint16_t* As) {
    const uint16_t* Bs = As + TA::ELEMS;
    constexpr int KS = MF == 32 ? 16 : 32;       // k per MFMA
#pragma unroll
    for (int s = 0; s < BK / KS; ++s) {
      h16x8 fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = load_frag<BM, BK, AKC, MF>(As, wr * WTM + i * MF, s);
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = load_frag<BN, BK, BKC, MF>(Bs, wc * WTN + j * MF, s);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if constexpr (MF == 32) acc[i][j] = mfma32(fb[j], fa[i], acc[i][j]);
          else acc[i][j] = mfma16(fb[j], fa[i], acc[i][j]);
        }
    }
  };
  const int nsteps = kbeg < kend ? (kend - kbeg + BK - 1) / BK : 0;
  if constexpr (GL) {
    // K-step i+1 is DMA'd into the other buffer while step i computes; the barrier at the end of
    // each step (its vmcnt(0) drains this wave's DMA) publishes it and retires the reads of the
    // buffer the next DMA overwrites.
    auto issue = [&](int k, uint16_t* dst) {
      if constexpr (GA) {
        uint4 unused[TA::PER_T];
        uint32_t okm;
        int ch;
        load_tile_gather_a<BM, BK, false, true>(p.cv, ccl, rg, k, kend, unused, ch, okm, dst);
      } else {
        la.dma(dst, k, kend);
      }
      lb.dma(dst + TA::ELEMS, k, kend);
    };
    // NS-stage ring: K-steps i+1 .. i+NS-1 are in flight while step i computes. Before the
    // barrier that publishes step i+1, a wave waits only for that step's DMAs (the newer ones
    // stay outstanding: loads complete in order, PER per step and thread).
    constexpr int PER = TA::PER_T + TB::PER_T;
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
      if (s < nsteps) issue(kbeg + s * BK, st + s * STAGE);
    dma_wait_barrier<NS, PER>(min(NS - 2, nsteps - 1));
    int cur = 0, nxt = NS - 1;
    for (int i = 0; i < nsteps; ++i) {
      if (i + NS - 1 < nsteps) issue(kbeg + (i + NS - 1) * BK, st + nxt * STAGE);
      compute(st + cur * STAGE);
      dma_wait_barrier<NS, PER>(min(NS - 2, nsteps - 2 - i));
      cur = cur + 1 == NS ? 0 : cur + 1;
      nxt = nxt + 1 == NS ? 0 : nxt + 1;
    }
  } else {
    if (nsteps > 0) {
      fetch(kbeg, R0);
      stage(st, R0);
    }
    __syncthreads();
    int cur = 0;
    for (int i = 0; i < nsteps; ++i) {
      const bool more = i + 1 < nsteps;
      if (more) fetch(kbeg + (i + 1) * BK, R0);
      compute(st + cur * STAGE);
      if (more) stage(st + (cur ^ 1) * STAGE, R0);
      __syncthreads();
      cur ^= 1;
    }
  }

  // ---- epilogue. B is the MFMA's first operand, so each accumulator holds Cᵀ: lane l has
  // MF = 16: C[m = .. + (l&15)][n = .. + 4*(l>>4) + r], r = 0..3 (four consecutive columns);
  // MF = 32: C[m = .. + (l&31)][n = .. + 8*g + 4*(l>>5) + r] in register 4g + r, g = 0..3.
  const int lm = l & (MF - 1), ln = MF == 32 ? 4 * (l >> 5) : 4 * (l >> 4);
  const bool bf_out = EPI != EPI_PARTIAL && p.out_bf16;
  static_assert(EPI != EPI_BSTATS || GA || CV == CV_NONE, "backward statistics: row outputs only");
  uint16_t* Ch = reinterpret_cast<uint16_t*>(lds);                  // bf16 tile [BM][LDH]
  float* red = reinterpret_cast<float*>(lds + BM * LDH * 2);        // stats [2 wave rows][2][BN]
  if (EPI != EPI_PARTIAL) {
    // bias / ReLU / rounding in registers; column statistics; bf16 staging of the whole tile
#pragma unroll
    for (int jg = 0; jg < FN * NG; ++jg) {
      const int j = jg / NG, g4 = jg % NG;
      const int nl = wc * WTN + j * MF + 8 * g4 + ln;
      const int n = n0 + nl;
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if (p.bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = n + r < p.N ? p.bias[n + r] : 0.f;
      }
      float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int ml = wr * WTM + i * MF + lm;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float x = acc[i][j][4 * g4 + r] + bv[r];
          if (p.relu) x = fmaxf(x, 0.f);
          v[r] = x;
        }
        if (bf_out) {
          uint16_t h[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            h[r] = f2h(v[r]);
            v[r] = h2f(h[r]);
          }
          *reinterpret_cast<uint2*>(Ch + ml * LDH + nl) =
              make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16));
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][4 * g4 + r] = v[r];
        }
        // column statistics of the stored values (bf16-rounded when the output is bf16), from
        // the accumulators: a per-lane sum over the FM row blocks, then a 16-lane butterfly
        if (EPI == EPI_STATS && m0 + ml < Mrow) {
#pragma unroll
          for (int r = 0; r < 4; ++r) { s1[r] += v[r]; s2[r] += v[r] * v[r]; }
        }
      }
      if (EPI == EPI_STATS) {
        // the MF rows held by lanes sharing the column run (one DPP row / one half-wave), fixed
        // pairing order
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s1[r] = MF == 32 ? sum32(s1[r]) : sum16(s1[r]);
          s2[r] = MF == 32 ? sum32(s2[r]) : sum16(s2[r]);
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
  // EPI_BSTATS sums come from the stored chunks during the store pass: a thread's chunks all
  // cover the same 8 columns (GT is a multiple of BN/8), so it sums them in registers and one
  // LDS fold per tile finishes the job. (EPI_STATS folds in registers above: summing the staged
  // tile here cost 35-58 % of a K <= 256 forward GEMM, profiles/r3/gemm_big_v3_stats.jsonl.)
  static_assert(GT % (BN / 8) == 0, "store chunks must keep their column per thread");
  float cs1[8], cs2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { cs1[k] = 0.f; cs2[k] = 0.f; }
  // EPI_BSTATS: this thread's 8 columns' mean (and mask affine) — fixed for the whole tile
  float bmu[8], bsc[8], bsh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { bmu[k] = 0.f; bsc[k] = 0.f; bsh[k] = 0.f; }
  if constexpr (EPI == EPI_BSTATS) {
    const int gn0 = n0 + (threadIdx.x % (BN / 8)) * 8;
    if (gn0 + 8 <= p.N) {           // (the host guarantees N % 8 == 0)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        bmu[k] = p.bst_mean[gn0 + k];
        bsc[k] = p.bst_bits ? 0.f : p.bst_scale[gn0 + k];
        bsh[k] = p.bst_bits ? 0.f : p.bst_shift[gn0 + k];
      }
    }
  }
  if (bf_out) {
    constexpr int NCH = BM * (BN / 8) / GT;          // store chunks per thread
    static_assert(BM * (BN / 8) % GT == 0, "store chunks must split evenly");
    const bool vec = (p.ldc & 7) == 0;
    // output row of a tile row (a parity class scatters its rows to its pixels)
    auto orow_of = [&](int gm) -> int64_t {
      if (GA && (p.cv.osy > 1 || p.cv.osx > 1)) {
        const int hw = ccl.Hg * ccl.Wg, b = gm / hw, rem = gm - b * hw;
        const int y = rem / ccl.Wg, x = rem - y * ccl.Wg;
        return ((int64_t)b * p.cv.Hout + y * p.cv.osy + ccl.py) * p.cv.Wout + x * p.cv.osx + ccl.px;
      }
      return gm;
    };
    // One chunk of the store pass: stats of the staged tile, addend, store, EPI_BSTATS sums.
    // `pa` / `px` / `pxb` are the chunk's prefetched addend, BN input and ReLU-bitmap byte.
    auto store_chunk = [&](int c, const uint4& pa, const uint4& px, uint32_t pxb, bool pref) {
      const int r = c / (BN / 8), cc = (c % (BN / 8)) * 8;
      const int gm = m0 + r, gn = n0 + cc;
      if (gm >= Mrow || gn >= p.N) return;
      const uint16_t* src = Ch + r * LDH + cc;
      const int64_t orow = orow_of(gm);
      uint16_t* dst = static_cast<uint16_t*>(p.C) + orow * p.ldc + gn;
      // the addend is aligned with the OUTPUT rows (a parity class adds into its own pixels,
      // e.g. a strided shortcut's data gradient accumulated into the block's dx in place)
      const int64_t aoff = orow * p.ldc + gn;
      if (vec && gn + 8 <= p.N) {
        uint4 v = *reinterpret_cast<const uint4*>(src);
        if (p.addend) v = add_h16x8(v, pref ? pa : masked_addend8(p.addend, p.add_bits, aoff));
        *reinterpret_cast<uint4*>(dst) = v;
        if constexpr (EPI == EPI_BSTATS) {
          // the stored gradient (bf16, as the BN backward would read it), masked by the ReLU of
          // that BN's output, against its input x at the same element
          const uint32_t w[4] = {v.x, v.y, v.z, v.w}, xw[4] = {px.x, px.y, px.z, px.w};
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float d = k & 1 ? hhi(w[k >> 1]) : hlo(w[k >> 1]);
            const float xv = k & 1 ? hhi(xw[k >> 1]) : hlo(xw[k >> 1]);
            const bool m = p.bst_bits ? ((pxb >> k) & 1u) != 0u : fmaf(xv, bsc[k], bsh[k]) > 0.f;
            const float dm = m ? d : 0.f;
            cs1[k] += dm;
            cs2[k] += dm * (xv - bmu[k]);
          }
        }
      } else {
        for (int k = 0; k < 8 && gn + k < p.N; ++k) {
          uint16_t h = src[k];
          if (p.addend)
            h = f2h(h2f(h) +
                         masked_addend1(p.addend, p.add_bits, aoff + k));
          dst[k] = h;
        }
      }
    };
    const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
    if constexpr (EPI == EPI_BSTATS) {
      // The memory operands of the chunks (addend, BN input x, ReLU bitmap) are loaded four
      // chunks at a time before those chunks are processed — the first group before the
      // barrier — so their latency overlaps instead of stalling every chunk in turn.
      constexpr int PG = NCH < 4 ? NCH : 4;
      static_assert(NCH % PG == 0, "prefetch groups");
      uint4 pa[PG], px[PG];
      uint32_t pxb[PG];
      auto prefetch = [&](int g) {
#pragma unroll
        for (int j = 0; j < PG; ++j) {
          const int c = threadIdx.x + (g * PG + j) * GT;
          const int gm = m0 + c / (BN / 8), gn = n0 + (c % (BN / 8)) * 8;
          const bool ok = vec && gm < Mrow && gn + 8 <= p.N;
          const int64_t aoff = ok ? orow_of(gm) * p.ldc + gn : 0;
          pa[j] = (ok && p.addend) ? masked_addend8(p.addend, p.add_bits, aoff) : z4;
          px[j] = ok ? *reinterpret_cast<const uint4*>(p.bst_x + aoff) : z4;
          pxb[j] = (ok && p.bst_bits) ? (uint32_t)p.bst_bits[aoff >> 3] : 0u;
        }
      };
      prefetch(0);
      __syncthreads();
#pragma unroll
      for (int g = 0; g < NCH / PG; ++g) {
        if (g > 0) prefetch(g);
#pragma unroll
        for (int j = 0; j < PG; ++j) store_chunk(threadIdx.x + (g * PG + j) * GT, pa[j], px[j], pxb[j], true);
      }
    } else {
      __syncthreads();
      for (int c = threadIdx.x; c < BM * (BN / 8); c += GT) store_chunk(c, z4, z4, 0u, false);
    }
  } else {
    // fp32 output or split-K slab: two halves through an fp32 staging tile
    float* Cs = reinterpret_cast<float*>(lds);
    float* P = EPI == EPI_PARTIAL ? p.partial + (int64_t)split * Mrow * p.N : nullptr;
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
#pragma unroll
            for (int g4 = 0; g4 < NG; ++g4)
              *reinterpret_cast<float4*>(Cs + (i * MF + lm) * LDC + wc * WTN + j * MF + 8 * g4 + ln) =
                  make_float4(acc[i][j][4 * g4], acc[i][j][4 * g4 + 1], acc[i][j][4 * g4 + 2],
                              acc[i][j][4 * g4 + 3]);
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
    // the two wave rows' column sums (red[], written before the store pass's barrier)
    for (int c = threadIdx.x; c < BN; c += GT) {
      const int n = n0 + c;
      if (n >= p.N) continue;
      const int srow = tm + (GA ? zc * tiles_m : 0);
      p.stats[(int64_t)srow * 2 * p.N + n] = red[0 * BN + c] + red[2 * BN + c];
      p.stats[(int64_t)srow * 2 * p.N + p.N + n] = red[1 * BN + c] + red[3 * BN + c];
    }
  }
  if (EPI == EPI_BSTATS) {
    // fold the per-thread column sums: GT/(BN/8) threads share each 8-column group
    constexpr int G8 = BN / 8, Q = GT / G8;
    // statistics row: the M-tile (+ the parity class: classes stack their tiles_m rows)
    const int srow = tm + (GA ? zc * tiles_m : 0);
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
      p.stats[(int64_t)srow * 2 * p.N + n] = a;
      p.stats[(int64_t)srow * 2 * p.N + p.N + n] = b;
    }
  }
}

}  // namespace lw
