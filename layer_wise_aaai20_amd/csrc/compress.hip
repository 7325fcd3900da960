// Gradient-compression kernels for gfx950 (MI355X, CDNA4, wave64).
//
// One launch (or one fixed chain of launches) handles ALL segments (= layers) of a communication
// bucket: the reference runs its compressor once per parameter tensor with torch ops
// (CIFAR10/core.py:175-215, IMAGENET/training/train_imagenet_nv.py:255-295; SURVEY.md §2.5
// N1-N9). Kernels here:
//
//   Top-K / Random-K (exact selection):
//     k_small_select   one workgroup per segment of <= 4096 elements: registers + LDS radix select
//                      + order-preserving compaction, EF fused.
//     k_hist<PASS>     multi-block 11/10/10-bit radix histogram passes for large segments
//                      (pass 0 fuses the error-feedback add g' = g + e).
//     k_select<PASS>   one workgroup per large segment: picks the digit holding the m-th largest key.
//     k_count, k_scan  per-block (gt, eq) counts and their per-segment exclusive scan.
//     k_write          order-preserving compaction into (index, value) pairs or index-free values,
//                      EF residual e = g' with the sent positions zeroed.
//   Threshold-v / adaptive threshold: k_partial + k_finalize (abs-max), k_thresh_state, then the
//                      same count / scan / write chain with "keep every key >= t".
//   TernGrad / QSGD:   k_partial + k_finalize (abs-max or L2 norm), k_quant (Philox dither, bit
//                      packing, EF), k_dequant (rank-ordered dequantise-and-average).
//   Unpack:            k_unpack_pairs (rank-ordered LDS accumulation of every rank's pairs for a
//                      4096-element chunk: deterministic and bit-identical on all ranks),
//                      k_unpack_validx (index-free Random-K).
//
// Selection keys are 31-bit: |x| bit patterns for Top-K/threshold (monotone in |x|), Philox hashes
// forced odd for Random-K (so padding/invalid keys of 0 never win).
#include "common.h"
#include "lw_kernels.h"
#include "elem16.h"
#include "sgd_elem.h"

#include <algorithm>
#include <cstdlib>

namespace lw {

constexpr int NT = 256;
#ifndef LW_HIST_CP
#define LW_HIST_CP 4             // interleaved LDS histogram copies in the first radix pass
#endif
static_assert((LW_HIST_CP & (LW_HIST_CP - 1)) == 0, "LW_HIST_CP: a power of two");
#ifndef LW_FUSED_SELECT
#define LW_FUSED_SELECT 1        // 0: the 9-launch chain (k_select per pass, k_count, k_fill_tail)
#endif
#ifndef LW_FW_SCAN_MAX
#define LW_FW_SCAN_MAX 512       // k_write sums its segment's earlier task counts up to this many
#endif
#ifndef LW_HIST_TPB
#define LW_HIST_TPB 4            // 8192-element tasks per histogram workgroup (see k_hist) once a
#endif                           // launch has LW_HIST_TPB_MIN tasks; 1 below that
#define LW_STR_(x) #x
#define LW_PRAGMA_UNROLL(n) _Pragma(LW_STR_(unroll n))
#ifndef LW_HIST_UNROLL
#define LW_HIST_UNROLL 2         // strides of NT*4 keys in flight per k_hist loop iteration
#endif
#ifndef LW_HIST_MC_FAST
#define LW_HIST_MC_FAST 1        // momentum-corrected pass 0 takes k_hist's batched-load path too
#endif
#ifndef LW_HIST_TPB_MIN
#define LW_HIST_TPB_MIN 2048
#endif
constexpr int EPB = kLargeEPB;       // elements per block in the multi-block passes (8192)
constexpr int EPT = EPB / NT;        // 32 contiguous elements per thread in k_write / k_quant
constexpr int SEPT = kSmallMax / NT; // 16 per thread in k_small_select
constexpr uint32_t SENT = 0x7fffffffu;
constexpr int HIST_WORDS = 4096;     // 2048 + 1024 + 1024 bins per large segment

__device__ __forceinline__ uint32_t abs_key(float x) { return __float_as_uint(x) & 0x7fffffffu; }

// Momentum correction of one element (optim.hip k_mc_prep, parallel/engine.py _mc_prologue):
// g' = g + wd·p, u = mc·u + g', returns u — every product and sum rounded on its own.
__device__ __forceinline__ float mc_step(float g, float& u, float p, float wd, float mc) {
#pragma clang fp contract(off)
  const float gw = wd != 0.f ? g + p * wd : g;
  u = u * mc + gw;
  return u;
}

__device__ __forceinline__ uint32_t randk_key(uint32_t i, uint32_t gid, uint32_t step, uint32_t s0,
                                              uint32_t s1) {
  const u4 r = philox4x32_10(u4{i >> 2, gid, step, 1u << 24}, s0, s1);
  return (pick(r, i & 3) >> 1) | 1u;
}

// group of 4 keys starting at a multiple of 4
__device__ __forceinline__ void randk_key4(uint32_t i0, uint32_t gid, uint32_t step, uint32_t s0,
                                           uint32_t s1, uint32_t k[4]) {
  const u4 r = philox4x32_10(u4{i0 >> 2, gid, step, 1u << 24}, s0, s1);
  k[0] = (r.x >> 1) | 1u; k[1] = (r.y >> 1) | 1u; k[2] = (r.z >> 1) | 1u; k[3] = (r.w >> 1) | 1u;
}

template <int PASS> struct PassCfg;
template <> struct PassCfg<0> { static constexpr int BITS = 11, SHIFT = 20, HOFF = 0; };
template <> struct PassCfg<1> { static constexpr int BITS = 10, SHIFT = 10, HOFF = 2048; };
template <> struct PassCfg<2> { static constexpr int BITS = 10, SHIFT = 0, HOFF = 3072; };

// Find the digit d holding the m-th largest key of histogram h (NB bins) and the rank of that key
// within bin d. Block-wide; all threads return the same values.
template <int NB, int TB = NT>
__device__ __forceinline__ void select_digit(const uint32_t* h, uint32_t m, uint32_t& d_out,
                                             uint32_t& m_out, uint32_t* arr /*TB*/,
                                             uint32_t* scr /*TB/WAVE*/, uint32_t* res /*2*/) {
  constexpr int BPT = NB / TB;
  const int j = threadIdx.x;
  uint32_t loc[BPT];
  uint32_t sum = 0;
#pragma unroll
  for (int b = 0; b < BPT; ++b) { loc[b] = h[j * BPT + b]; sum += loc[b]; }
  if (j == 0) { res[0] = 0; res[1] = m; }
  arr[TB - 1 - j] = sum;
  __syncthreads();
  uint32_t tot;
  const uint32_t e = block_excl_scan<TB>(arr[j], scr, tot);
  arr[j] = e;
  __syncthreads();
  const uint32_t above = arr[TB - 1 - j];   // keys in bins above this thread's range
  if (above < m && m <= above + sum) {
    uint32_t cum = above;
#pragma unroll
    for (int b = BPT - 1; b >= 0; --b) {
      if (cum + loc[b] >= m) { res[0] = j * BPT + b; res[1] = m - cum; break; }
      cum += loc[b];
    }
  }
  __syncthreads();
  d_out = res[0];
  m_out = res[1];
  __syncthreads();
}

// Final per-segment decision shared by the small and large paths.
__device__ __forceinline__ void finish_state(SelState& s, int km, uint32_t keep, uint32_t m_rem,
                                             uint32_t eq_total, uint32_t cap) {
  s.cnt_gt = keep - m_rem;
  if (km == KM_RANDK) {
    s.quota = m_rem;                       // exactly `keep` elements, ties broken by index
  } else {
    // Top-K keeps every tie (core.py:182 `|g| < thr` zeroed) up to the payload capacity;
    // zero-valued ties carry nothing and are never sent.
    const uint32_t room = cap > s.cnt_gt ? cap - s.cnt_gt : 0u;
    s.quota = s.tkey == 0 ? 0u : min(eq_total, room);
  }
  s.total = s.cnt_gt + s.quota;
  s.cap = cap;
}

// ------------------------------------------------------------------------------------------
// Small segments: whole selection + compaction in one workgroup.
// ------------------------------------------------------------------------------------------
template <int KM, int OUT, bool EF, bool MC = false>
__global__ __launch_bounds__(NT) void k_small_select(
    float* __restrict__ g, float* __restrict__ ef, const int64_t* __restrict__ seg_off,
    const int32_t* __restrict__ seg_n, const int32_t* __restrict__ keep,
    const int64_t* __restrict__ cap_off, const int32_t* __restrict__ small_segs,
    int2* __restrict__ pairs, float* __restrict__ vals, int32_t* __restrict__ idx_out,
    SelState* __restrict__ st_small, uint32_t gid_base, uint32_t step_arg, uint32_t s0, uint32_t s1, const uint32_t* __restrict__ stepp,
    unsigned long long* __restrict__ overflow, float* __restrict__ mom, McArgs mcx = McArgs{}) {
  // graph-captured steps read the step counter from device memory (csrc/lw_kernels.h)
  const uint32_t step = stepp != nullptr ? *stepp : step_arg;
  __shared__ uint32_t h[2048];
  __shared__ uint32_t arr[NT];
  __shared__ uint32_t scr[NT / WAVE];
  __shared__ uint32_t res[2];
  const int s = small_segs[blockIdx.x];
  const int n = seg_n[s];
  const int64_t off = seg_off[s];
  const uint32_t m = (uint32_t)keep[s];
  const int64_t c0 = cap_off[s];
  const uint32_t cap = (uint32_t)(cap_off[s + 1] - c0);
  float* gp = g + off;
  float* ep = EF ? ef + off : nullptr;
  const int base = threadIdx.x * SEPT;

  float v[SEPT];
  uint32_t key[SEPT];
  // fused momentum correction (McArgs): the compressor sees u = mc·u + g'
  float* up = MC ? mcx.u + off : nullptr;
  const float* pw = MC && mcx.p != nullptr ? mcx.p + off : nullptr;
  const float wd = MC && mcx.wd != nullptr ? mcx.wd[s] * mcx.wmul : 0.f;
#pragma unroll
  for (int k = 0; k < SEPT; ++k) {
    const int i = base + k;
    float x = 0.f;
    if (i < n) {
      x = gp[i];
      if (MC) {
        float u = up[i];
        x = mc_step(x, u, pw != nullptr ? pw[i] : 0.f, wd, mcx.mc);
        up[i] = u;
      }
      if (EF) x += ep[i];
    }
    v[k] = x;
  }
  if (KM == KM_TOPK) {
#pragma unroll
    for (int k = 0; k < SEPT; ++k) key[k] = (base + k < n) ? abs_key(v[k]) : 0u;
  } else {
#pragma unroll
    for (int k = 0; k < SEPT; k += 4) {
      uint32_t q[4];
      randk_key4(base + k, gid_base + s, step, s0, s1, q);
#pragma unroll
      for (int t = 0; t < 4; ++t) key[k + t] = (base + k + t < n) ? q[t] : 0u;
    }
  }

  // three radix passes over the register-resident keys
  uint32_t prefix = 0, mr = m;
  uint32_t eq_total = 0;
#pragma unroll
  for (int pass = 0; pass < 3; ++pass) {
    const int bits = pass == 0 ? 11 : 10;
    const int shift = pass == 0 ? 20 : (pass == 1 ? 10 : 0);
    const int nb = 1 << bits;
    for (int b = threadIdx.x; b < nb; b += NT) h[b] = 0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < SEPT; ++k) {
      if (base + k < n && (key[k] >> (shift + bits)) == prefix)
        atomicAdd(&h[(key[k] >> shift) & (nb - 1)], 1u);
    }
    __syncthreads();
    uint32_t d, mn;
    if (pass == 0) select_digit<2048>(h, mr, d, mn, arr, scr, res);
    else select_digit<1024>(h, mr, d, mn, arr, scr, res);
    if (pass == 2) eq_total = h[d];
    __syncthreads();
    prefix = (prefix << bits) | d;
    mr = mn;
  }
  SelState S;
  S.tkey = prefix;
  finish_state(S, KM, m, mr, eq_total, cap);
  if (threadIdx.x == 0) {
    st_small[blockIdx.x] = S;
    // ties the reference's `>=` rule keeps but the payload slack could not hold (left in EF)
    if (KM == KM_TOPK && overflow != nullptr && S.tkey != 0 && eq_total > S.quota)
      atomicAdd(overflow, (unsigned long long)(eq_total - S.quota));
  }

  // order-preserving compaction: (gt, eq) counts packed in one word (<= 4096 each)
  uint32_t cg = 0, ce = 0;
#pragma unroll
  for (int k = 0; k < SEPT; ++k) {
    if (base + k < n) { cg += key[k] > S.tkey; ce += key[k] == S.tkey; }
  }
  uint32_t tot;
  const uint32_t pre = block_excl_scan<NT>(cg | (ce << 16), scr, tot);
  uint32_t gb = pre & 0xffffu, eb = pre >> 16;
#pragma unroll
  for (int k = 0; k < SEPT; ++k) {
    const int i = base + k;
    if (i >= n) break;
    bool sel = false;
    uint32_t pos = 0;
    if (key[k] > S.tkey) { sel = true; pos = gb + min(eb, S.quota); ++gb; }
    else if (key[k] == S.tkey) { if (eb < S.quota) { pos = gb + eb; sel = pos < S.cap; } ++eb; }
    if (sel) {
      if (OUT == OUT_PAIRS) pairs[c0 + pos] = make_int2(i, __float_as_int(v[k]));
      else { vals[c0 + pos] = v[k]; idx_out[c0 + pos] = i; }
    }
    if (EF) ep[i] = sel ? 0.f : v[k];
    // momentum factor masking (DGC): a sent coordinate restarts its velocity, unless the whole
    // segment was sent (it then keeps ordinary momentum)
    if (mom != nullptr && sel && S.total < (uint32_t)n) mom[off + i] = 0.f;
  }
  if (OUT == OUT_PAIRS)
    for (uint32_t p = S.total + threadIdx.x; p < cap; p += NT) pairs[c0 + p] = make_int2(SENT, 0);
}

// ------------------------------------------------------------------------------------------
// Large segments: multi-block radix select.
// Coalesced layout for histogram/count passes: element = begin + j*NT*4 + tid*4 + {0..3}.
// ------------------------------------------------------------------------------------------
template <int KM, bool EFADD, bool MC = false>
__device__ __forceinline__ void load4_keys(float* gp, const float* ep, int i0, int end, uint32_t gid,
                                           uint32_t step, uint32_t s0, uint32_t s1, uint32_t k[4],
                                           bool valid[4], float* up = nullptr,
                                           const float* pp = nullptr, float wd = 0.f,
                                           float mc = 0.f) {
#pragma unroll
  for (int t = 0; t < 4; ++t) valid[t] = i0 + t < end;
  if (KM == KM_RANDK) {
    randk_key4(i0, gid, step, s0, s1, k);
    return;
  }
  // MC: the first pass turns g into the velocity u = mc·u + g' (stored to u) and, with EF, into
  // u + e — stored back to g either way, so the later passes read what the compressor sees
  float4 v;
  if (i0 + 3 < end) {
    v = *reinterpret_cast<const float4*>(gp + i0);
    if (MC) {
      float4 u = *reinterpret_cast<const float4*>(up + i0);
      float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
      if (pp != nullptr) p = *reinterpret_cast<const float4*>(pp + i0);
      v.x = mc_step(v.x, u.x, p.x, wd, mc); v.y = mc_step(v.y, u.y, p.y, wd, mc);
      v.z = mc_step(v.z, u.z, p.z, wd, mc); v.w = mc_step(v.w, u.w, p.w, wd, mc);
      *reinterpret_cast<float4*>(up + i0) = u;
    }
    if (EFADD) {
      const float4 e = *reinterpret_cast<const float4*>(ep + i0);
      v.x += e.x; v.y += e.y; v.z += e.z; v.w += e.w;
    }
    if (EFADD || MC) *reinterpret_cast<float4*>(gp + i0) = v;
  } else {
    float t4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (valid[t]) {
        float x = gp[i0 + t];
        if (MC) {
          float u = up[i0 + t];
          x = mc_step(x, u, pp != nullptr ? pp[i0 + t] : 0.f, wd, mc);
          up[i0 + t] = u;
        }
        if (EFADD) x += ep[i0 + t];
        if (EFADD || MC) gp[i0 + t] = x;
        t4[t] = x;
      }
    v = make_float4(t4[0], t4[1], t4[2], t4[3]);
  }
  k[0] = abs_key(v.x); k[1] = abs_key(v.y); k[2] = abs_key(v.z); k[3] = abs_key(v.w);
}

// Fused radix chain (FUSED = true, passes 1 and 2): a workgroup reaching a segment redoes the
// previous pass's digit selection itself, from that pass's complete integer histogram, instead of
// a k_select launch of its own — every workgroup derives the identical digit. The workgroup that
// holds the segment's first task publishes it (SelState p0/m0 after pass 0, p1/m1 after pass 1)
// for the next launch; no workgroup of this launch reads those fields.
template <int PASS, int TB = NT>
__device__ __forceinline__ void fused_prev_select(const uint32_t* __restrict__ hist_all,
                                                  SelState* __restrict__ st,
                                                  const int32_t* __restrict__ keep, int li, int s,
                                                  bool publish, uint32_t& prefix, uint32_t* arr,
                                                  uint32_t* scr, uint32_t* res) {
  const uint32_t* hb = hist_all + (size_t)li * HIST_WORDS;
  uint32_t d, mn;
  if constexpr (PASS == 1) {
    select_digit<2048, TB>(hb + PassCfg<0>::HOFF, (uint32_t)keep[s], d, mn, arr, scr, res);
    prefix = d;
    if (publish && threadIdx.x == 0) { st[li].p0 = prefix; st[li].m0 = mn; }
  } else {
    const uint32_t p0 = st[li].p0;
    select_digit<1024, TB>(hb + PassCfg<1>::HOFF, st[li].m0, d, mn, arr, scr, res);
    prefix = (p0 << PassCfg<1>::BITS) | d;
    if (publish && threadIdx.x == 0) { st[li].p1 = prefix; st[li].m1 = mn; }
  }
}

template <int KM, int PASS, bool EFADD, bool FUSED = false, bool MC = false, int TB = NT>
__global__ __launch_bounds__(TB) void k_hist(float* __restrict__ g, const float* __restrict__ ef,
                                             const int64_t* __restrict__ seg_off,
                                             const int32_t* __restrict__ seg_n,
                                             const int32_t* __restrict__ large_segs,
                                             const int2* __restrict__ tasks, int ntasks, int tpb,
                                             SelState* __restrict__ st,
                                             uint32_t* __restrict__ hist_all, uint32_t gid_base,
                                             uint32_t step_arg, uint32_t s0, uint32_t s1, const uint32_t* __restrict__ stepp,
                                             const int32_t* __restrict__ keep = nullptr,
                                             const int32_t* __restrict__ task_lo = nullptr,
                                             McArgs mcx = McArgs{}) {
  // graph-captured steps read the step counter from device memory (csrc/lw_kernels.h)
  const uint32_t step = stepp != nullptr ? *stepp : step_arg;
  using C = PassCfg<PASS>;
  constexpr int NB = 1 << C::BITS;
  // Pass 0 counts EVERY key, and gradient magnitudes cluster in a few exponent bins, so many
  // lanes of one ds_add hit the same word and serialise. CP interleaved copies of the histogram
  // (copy = lane % CP, bin-major so a bin's copies sit in adjacent banks) split those lanes;
  // passes 1/2 count only the keys under the selected prefix and keep one copy.
  constexpr int CP = PASS == 0 ? LW_HIST_CP : 1;
  static_assert(!FUSED || PASS > 0, "pass 0 has no previous selection");
  static_assert(EPB % (TB * 4) == 0, "whole strides per task");
  __shared__ uint32_t h[NB * CP];
  __shared__ uint32_t sarr[FUSED ? TB : 1], sscr[TB / WAVE], sres[2];
  // A workgroup takes `tpb` consecutive tasks (LW_HIST_TPB on large launches): zeroing the LDS
  // histogram (NB * CP words) and merging it into the segment's global one cost about as much LDS
  // traffic as counting one task's 8192 keys, so they are paid once per segment run of the
  // workgroup's tasks, not per task; a small launch keeps one task per workgroup so that it
  // still spreads over the CUs. Integer counts: the result does not depend on the grouping.
  // tpb < 0: the other way round, -tpb workgroups per task (a small launch spread over 4x the
  // workgroups; each takes its share of the task's strides)
  const int split = tpb < 0 ? -tpb : 1, per = tpb > 0 ? tpb : 1;
  const int ta = (int)(blockIdx.x / split) * per, tb = min(ntasks, ta + per);
  const int q_sub = (int)(blockIdx.x % split);
  auto flush = [&](int li) {
    uint32_t* gh = hist_all + (size_t)li * HIST_WORDS + C::HOFF;
    for (int b = threadIdx.x; b < NB; b += TB) {
      uint32_t c = 0;
#pragma unroll
      for (int j = 0; j < CP; ++j) c += h[b * CP + j];
      if (c) atomicAdd(gh + b, c);
    }
  };
  // Exact zeros (a ReLU / dropout layer's weight gradient is full of them: VGG-16's 103 M-weight
  // classifier input) all land in bin 0 and would serialise every wave's LDS atomic on one word;
  // a thread counts them in a register and adds its count once per segment run (Top-K keys only:
  // Random-K keys are odd, never 0).
  uint32_t zc = 0;
  auto add_zeros = [&]() {
    if (zc) atomicAdd(&h[threadIdx.x & (CP - 1)], zc);
    zc = 0;
  };
  int cur = -1;
  uint32_t prefix = 0u;
  for (int ti = ta; ti < tb; ++ti) {
    const int2 t = tasks[ti];
    const int li = t.x, begin = t.y;
    if (li != cur) {                     // (uniform: the whole workgroup switches segment)
      if (cur >= 0) {
        add_zeros();
        __syncthreads();
        flush(cur);
      }
      __syncthreads();
      for (int b = threadIdx.x; b < NB * CP; b += TB) h[b] = 0;
      cur = li;
      if constexpr (FUSED)
        fused_prev_select<PASS, TB>(hist_all, st, keep, li, large_segs[li],
                                ti == task_lo[li] && q_sub == 0, prefix, sarr, sscr, sres);
      else
        prefix = PASS > 0 ? st[li].prefix : 0u;
      __syncthreads();
    }
    const int s = large_segs[li];
    const int n = seg_n[s];
    const int64_t off = seg_off[s];
    float* gp = g + off;
    const float* ep = EFADD ? ef + off : nullptr;
    const int end = min(begin + EPB, n);
    float* up = MC ? mcx.u + off : nullptr;
    const float* pw = MC && mcx.p != nullptr ? mcx.p + off : nullptr;
    const float wd = MC && mcx.wd != nullptr ? mcx.wd[s] * mcx.wmul : 0.f;
    const int nstr = EPB / (TB * 4) / split;          // strides of TB*4 keys for this workgroup
    // four consecutive keys with one digit (a replicated layer's gradient — VGG-16 fc1 repeats
    // each value 49 times — or a flat region) are counted with one atomic
    auto count4 = [&](const uint32_t k[4], const bool valid[4]) {
      uint32_t bin[4];
      bool in[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        in[q] = valid[q] && (k[q] >> (C::SHIFT + C::BITS)) == prefix;
        if (KM != KM_RANDK && in[q] && k[q] == 0u) { ++zc; in[q] = false; }
        bin[q] = (k[q] >> C::SHIFT) & (NB - 1);
      }
      uint32_t* hb = h + (threadIdx.x & (CP - 1));
      if (in[0] && in[1] && in[2] && in[3] && bin[0] == bin[1] && bin[1] == bin[2] &&
          bin[2] == bin[3]) {
        atomicAdd(hb + bin[0] * CP, 4u);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (in[q]) atomicAdd(hb + bin[q] * CP, 1u);
      }
    };
    const int j0 = q_sub * nstr;
    if (KM != KM_RANDK && (!MC || LW_HIST_MC_FAST) && begin + (j0 + nstr) * TB * 4 <= end) {
      // Every stride of this workgroup in bounds (all but a segment's last task): issue all its
      // loads before the first use — up to 8 float4 per operand in flight per thread instead of
      // the loop's 2, which a data-dependent bound keeps from being hoisted. One workgroup per CU
      // (a 276-task entire-model bucket) was latency-bound at 2 strides in flight.
      constexpr int MS = EPB / (TB * 4);
      // momentum correction streams four operands: two batches of half the strides keep it
      // below 256 VGPRs
      constexpr int BATCH = MC && MS > 1 ? MS / 2 : MS;
      // (no early exit in these loops: they must unroll fully so the arrays stay in registers)
#pragma unroll
      for (int h = 0; h < MS; h += BATCH) {
        float4 gv[BATCH], ev[BATCH], uv[BATCH], pv[BATCH];
#pragma unroll
        for (int jj = 0; jj < BATCH; ++jj) {
          const int j = h + jj;
          if (j < nstr) {
            const int i0 = begin + (j0 + j) * TB * 4 + threadIdx.x * 4;
            gv[jj] = *reinterpret_cast<const float4*>(gp + i0);
            if (EFADD) ev[jj] = *reinterpret_cast<const float4*>(ep + i0);
            if (MC) {
              uv[jj] = *reinterpret_cast<const float4*>(up + i0);
              pv[jj] = pw != nullptr ? *reinterpret_cast<const float4*>(pw + i0)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
            }
          }
        }
#pragma unroll
        for (int jj = 0; jj < BATCH; ++jj) {
          const int j = h + jj;
          if (j >= nstr) continue;
          const int i0 = begin + (j0 + j) * TB * 4 + threadIdx.x * 4;
          float4 v = gv[jj];
          if (MC) {
            const float mc = mcx.mc;
            float4 u = uv[jj];
            v.x = mc_step(v.x, u.x, pv[jj].x, wd, mc); v.y = mc_step(v.y, u.y, pv[jj].y, wd, mc);
            v.z = mc_step(v.z, u.z, pv[jj].z, wd, mc); v.w = mc_step(v.w, u.w, pv[jj].w, wd, mc);
            *reinterpret_cast<float4*>(up + i0) = u;
          }
          if (EFADD) { v.x += ev[jj].x; v.y += ev[jj].y; v.z += ev[jj].z; v.w += ev[jj].w; }
          if (EFADD || MC) *reinterpret_cast<float4*>(gp + i0) = v;
          const uint32_t k[4] = {abs_key(v.x), abs_key(v.y), abs_key(v.z), abs_key(v.w)};
          const bool valid[4] = {true, true, true, true};
          count4(k, valid);
        }
      }
      continue;
    }
    LW_PRAGMA_UNROLL(LW_HIST_UNROLL)
    for (int j = j0; j < j0 + nstr; ++j) {
      const int i0 = begin + j * TB * 4 + threadIdx.x * 4;
      if (i0 >= end) break;
      uint32_t k[4];
      bool valid[4];
      load4_keys<KM, EFADD, MC>(gp, ep, i0, end, gid_base + s, step, s0, s1, k, valid, up, pw,
                                wd, MC ? mcx.mc : 0.f);
      count4(k, valid);
    }
  }
  add_zeros();
  __syncthreads();
  if (cur >= 0) flush(cur);
}

template <int KM, int PASS>
__global__ __launch_bounds__(NT) void k_select(const uint32_t* __restrict__ hist_all,
                                               SelState* __restrict__ st,
                                               const int32_t* __restrict__ large_segs,
                                               const int32_t* __restrict__ keep,
                                               const int64_t* __restrict__ cap_off,
                                               unsigned long long* __restrict__ overflow) {
  using C = PassCfg<PASS>;
  constexpr int NB = 1 << C::BITS;
  __shared__ uint32_t arr[NT];
  __shared__ uint32_t scr[NT / WAVE];
  __shared__ uint32_t res[2];
  const int li = blockIdx.x;
  const int s = large_segs[li];
  const uint32_t* h = hist_all + (size_t)li * HIST_WORDS + C::HOFF;
  const uint32_t m = PASS == 0 ? (uint32_t)keep[s] : st[li].m;
  const uint32_t prefix = PASS == 0 ? 0u : st[li].prefix;
  uint32_t d, mn;
  select_digit<NB>(h, m, d, mn, arr, scr, res);
  if (threadIdx.x == 0) {
    SelState S = st[li];
    S.prefix = (prefix << C::BITS) | d;
    S.m = mn;
    if (PASS == 2) {
      S.tkey = S.prefix;
      finish_state(S, KM, (uint32_t)keep[s], mn, h[d], (uint32_t)(cap_off[s + 1] - cap_off[s]));
      if (KM == KM_TOPK && overflow != nullptr && S.tkey != 0 && h[d] > S.quota)
        atomicAdd(overflow, (unsigned long long)(h[d] - S.quota));
    }
    st[li] = S;
  }
}

// Threshold methods: t = key(V) (Thresholdv) or key(max|g|/2) (AdaptiveThreshold); keep all ties.
__global__ void k_thresh_state(SelState* __restrict__ st, const float* __restrict__ segmax,
                               int nseg, float V, int adaptive) {
  const int li = blockIdx.x * blockDim.x + threadIdx.x;
  if (li >= nseg) return;
  const float thr = adaptive ? segmax[li] * 0.5f : V;
  SelState S{};
  S.tkey = abs_key(thr);
  S.cnt_gt = 0;
  S.quota = S.tkey == 0 ? 0u : 0xffffffffu;
  st[li] = S;
}

template <int KM, bool EFADD>
__global__ __launch_bounds__(NT) void k_count(float* __restrict__ g, const float* __restrict__ ef,
                                              const int64_t* __restrict__ seg_off,
                                              const int32_t* __restrict__ seg_n,
                                              const int32_t* __restrict__ large_segs,
                                              const int2* __restrict__ tasks,
                                              const SelState* __restrict__ st,
                                              uint2* __restrict__ cnt, uint32_t gid_base,
                                              uint32_t step_arg, uint32_t s0, uint32_t s1, const uint32_t* __restrict__ stepp) {
  // graph-captured steps read the step counter from device memory (csrc/lw_kernels.h)
  const uint32_t step = stepp != nullptr ? *stepp : step_arg;
  __shared__ uint32_t scr[NT / WAVE];
  const int2 t = tasks[blockIdx.x];
  const int li = t.x, begin = t.y;
  const int s = large_segs[li];
  const int n = seg_n[s];
  const int64_t off = seg_off[s];
  const uint32_t tk = st[li].tkey;
  float* gp = g + off;
  const float* ep = EFADD ? ef + off : nullptr;
  const int end = min(begin + EPB, n);
  uint32_t cg = 0, ce = 0;
#pragma unroll 2
  for (int j = 0; j < EPB / (NT * 4); ++j) {
    const int i0 = begin + j * NT * 4 + threadIdx.x * 4;
    if (i0 >= end) break;
    uint32_t k[4];
    bool valid[4];
    load4_keys<KM, EFADD>(gp, ep, i0, end, gid_base + s, step, s0, s1, k, valid);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (valid[q]) { cg += k[q] > tk; ce += k[q] == tk; }
  }
  uint32_t tg, te;
  block_excl_scan<NT>(cg, scr, tg);
  block_excl_scan<NT>(ce, scr, te);
  if (threadIdx.x == 0) cnt[blockIdx.x] = make_uint2(tg, te);
}

// Fused chain: the pass-2 digit selection and finish_state (k_select<2>) in every workgroup at a
// segment switch, then the per-task (gt, eq) counts of k_count for `tpb` tasks per workgroup.
// The workgroup holding the segment's first task publishes the final state (and counts the
// Top-K ties that did not fit) for k_scan / k_write.
template <int KM>
__global__ __launch_bounds__(NT) void k_count_sel(float* __restrict__ g,
                                                  const int64_t* __restrict__ seg_off,
                                                  const int32_t* __restrict__ seg_n,
                                                  const int32_t* __restrict__ large_segs,
                                                  const int2* __restrict__ tasks, int ntasks,
                                                  int tpb, const int32_t* __restrict__ task_lo,
                                                  SelState* __restrict__ st,
                                                  const uint32_t* __restrict__ hist_all,
                                                  const int32_t* __restrict__ keep,
                                                  const int64_t* __restrict__ cap_off,
                                                  unsigned long long* __restrict__ overflow,
                                                  uint2* __restrict__ cnt, uint32_t gid_base,
                                                  uint32_t step_arg, uint32_t s0, uint32_t s1,
                                                  const uint32_t* __restrict__ stepp) {
  const uint32_t step = stepp != nullptr ? *stepp : step_arg;
  __shared__ uint32_t arr[NT], scr[NT / WAVE], res[2];
  const int split = tpb < 0 ? -tpb : 1, per = tpb > 0 ? tpb : 1;     // (as k_hist)
  const int ta = (int)(blockIdx.x / split) * per, tb = min(ntasks, ta + per);
  const int q_sub = (int)(blockIdx.x % split);
  int cur = -1;
  uint32_t tk = 0;
  for (int ti = ta; ti < tb; ++ti) {
    const int2 t = tasks[ti];
    const int li = t.x, begin = t.y;
    const int s = large_segs[li];
    if (li != cur) {                     // (uniform across the workgroup)
      cur = li;
      const uint32_t* h = hist_all + (size_t)li * HIST_WORDS + PassCfg<2>::HOFF;
      const uint32_t p1 = st[li].p1;
      uint32_t d, mn;
      select_digit<1024>(h, st[li].m1, d, mn, arr, scr, res);
      SelState S;
      S.prefix = (p1 << PassCfg<2>::BITS) | d;
      S.m = mn;
      S.tkey = S.prefix;
      const uint32_t hd = h[d];
      finish_state(S, KM, (uint32_t)keep[s], mn, hd, (uint32_t)(cap_off[s + 1] - cap_off[s]));
      tk = S.tkey;
      if (ti == task_lo[li] && q_sub == 0 && threadIdx.x == 0) {
        SelState& o = st[li];
        o.prefix = S.prefix; o.m = S.m; o.tkey = S.tkey; o.quota = S.quota;
        o.cnt_gt = S.cnt_gt; o.total = S.total; o.cap = S.cap;
        if (KM == KM_TOPK && overflow != nullptr && S.tkey != 0 && hd > S.quota)
          atomicAdd(overflow, (unsigned long long)(hd - S.quota));
      }
    }
    const int n = seg_n[s];
    const int64_t off = seg_off[s];
    float* gp = g + off;
    const int end = min(begin + EPB, n);
    // (gt, eq) per sub-task of EPB / kWriteSub elements, packed gt | eq << 16 (each <= 2048)
    constexpr int STRIDES = EPB / (NT * 4), PER_SUB = STRIDES / kWriteSub;
    static_assert(PER_SUB >= 1 && STRIDES % kWriteSub == 0, "sub-task = whole strides");
    uint32_t c[kWriteSub];
#pragma unroll
    for (int q = 0; q < kWriteSub; ++q) c[q] = 0;
    // split == kWriteSub: this workgroup counts sub-task q_sub only
    const int jlo = split > 1 ? q_sub * PER_SUB : 0, jhi = split > 1 ? jlo + PER_SUB : STRIDES;
    if (KM != KM_RANDK && begin + jhi * NT * 4 <= end) {
      // all of this workgroup's strides in bounds: every load issued before the first compare
      // (as k_hist's fast path)
      float4 gv[STRIDES];
#pragma unroll
      for (int j = 0; j < STRIDES; ++j)
        if (j >= jlo && j < jhi)
          gv[j] = *reinterpret_cast<const float4*>(gp + begin + j * NT * 4 + threadIdx.x * 4);
#pragma unroll
      for (int j = 0; j < STRIDES; ++j) {
        if (j < jlo || j >= jhi) continue;
        const uint32_t k[4] = {abs_key(gv[j].x), abs_key(gv[j].y), abs_key(gv[j].z),
                               abs_key(gv[j].w)};
#pragma unroll
        for (int q = 0; q < 4; ++q)
          c[j / PER_SUB] += (k[q] > tk ? 1u : 0u) + (k[q] == tk ? 0x10000u : 0u);
      }
    } else {
#pragma unroll
      for (int j = 0; j < STRIDES; ++j) {
        const int i0 = begin + j * NT * 4 + threadIdx.x * 4;
        if (j < jlo || j >= jhi || i0 >= end) continue;
        uint32_t k[4];
        bool valid[4];
        load4_keys<KM, false>(gp, nullptr, i0, end, gid_base + s, step, s0, s1, k, valid);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (valid[q]) c[j / PER_SUB] += (k[q] > tk ? 1u : 0u) + (k[q] == tk ? 0x10000u : 0u);
      }
    }
#pragma unroll
    for (int q = 0; q < kWriteSub; ++q) {
      if (split > 1 && q != q_sub) continue;        // (uniform)
      uint32_t tot;
      block_excl_scan<NT>(c[q], scr, tot);
      if (threadIdx.x == 0) cnt[ti * kWriteSub + q] = make_uint2(tot & 0xffffu, tot >> 16);
    }
    __syncthreads();                     // scr / arr reuse by the next task
  }
}

// One workgroup per large segment: exclusive scan of the per-block (gt, eq) counts.
template <int KM>
__global__ __launch_bounds__(NT) void k_scan(const uint2* __restrict__ cnt, uint2* __restrict__ pre,
                                             const int32_t* __restrict__ task_lo,
                                             SelState* __restrict__ st,
                                             int32_t* __restrict__ count_out, int sub = 1) {
  __shared__ uint32_t scr[NT / WAVE];
  const int li = blockIdx.x;
  const int lo = task_lo[li] * sub, hi = task_lo[li + 1] * sub;   // (sub-tasks per task)
  // A thread owns SV consecutive entries per tile of NT * SV: one pair of block scans per tile
  // instead of per NT entries (VGG-16's 103 M-weight layer has 50 k sub-task entries: 196 serial
  // scan rounds took 0.2 ms a step; 25 now).
  constexpr int SV = 8;
  uint32_t carry_g = 0, carry_e = 0;
  for (int b = lo; b < hi; b += NT * SV) {
    const int i0 = b + (int)threadIdx.x * SV;
    uint2 c[SV];
    uint32_t sg = 0, se = 0;
#pragma unroll
    for (int v = 0; v < SV; ++v) {
      c[v] = i0 + v < hi ? cnt[i0 + v] : make_uint2(0, 0);
      sg += c[v].x;
      se += c[v].y;
    }
    uint32_t tg, te;
    uint32_t eg = block_excl_scan<NT>(sg, scr, tg) + carry_g;
    uint32_t ee = block_excl_scan<NT>(se, scr, te) + carry_e;
#pragma unroll
    for (int v = 0; v < SV; ++v) {
      if (i0 + v < hi) pre[i0 + v] = make_uint2(eg, ee);
      eg += c[v].x;
      ee += c[v].y;
    }
    carry_g += tg;
    carry_e += te;
  }
  if (threadIdx.x == 0) {
    SelState S = st[li];
    if (KM == KM_THRESH) {
      S.cnt_gt = carry_g;
      S.quota = S.tkey == 0 ? 0u : carry_e;
      S.total = S.cnt_gt + S.quota;
      st[li] = S;
    }
    if (count_out) count_out[li] = (int32_t)S.total;
  }
}

// Threshold methods on the reference's dense wire: the bucket is overwritten in place with its
// compressed dense vector (kept entries, zeros elsewhere) and the residual goes to EF — no counts,
// no payload sizing, so no host round trip in the middle of backward. EFADD: g += ef first (not
// yet folded in by k_partial); EFW: write the residual.
template <bool EFADD, bool EFW>
__global__ __launch_bounds__(NT) void k_thresh_dense(float* __restrict__ g, float* __restrict__ ef,
                                                     const int64_t* __restrict__ seg_off,
                                                     const int32_t* __restrict__ seg_n,
                                                     const int32_t* __restrict__ large_segs,
                                                     const int2* __restrict__ tasks,
                                                     const SelState* __restrict__ st) {
  const int2 t = tasks[blockIdx.x];
  const int li = t.x, begin = t.y;
  const int s = large_segs[li];
  const int n = seg_n[s];
  const int64_t off = seg_off[s];
  const uint32_t tk = st[li].tkey;
  const int end = min(begin + EPB, n);
  float* gp = g + off;
  float* ep = EFW ? ef + off : nullptr;
  for (int i = begin + threadIdx.x; i < end; i += NT) {
    float x = gp[i];
    if (EFADD) x += ep[i];
    const uint32_t k = abs_key(x);
    const bool keep = tk != 0 ? k >= tk : k > 0;
    gp[i] = keep ? x : 0.f;
    if (EFW) ep[i] = keep ? 0.f : x;
  }
}

// Per-segment capacity for the threshold path is only known after the count exchange.
__global__ void k_set_caps(SelState* __restrict__ st, const int64_t* __restrict__ cap_off,
                           const int32_t* __restrict__ large_segs, int nseg,
                           unsigned long long* __restrict__ overflow) {
  const int li = blockIdx.x * blockDim.x + threadIdx.x;
  if (li >= nseg) return;
  const int s = large_segs[li];
  SelState S = st[li];
  S.cap = (uint32_t)(cap_off[s + 1] - cap_off[s]);
  if (S.total > S.cap) {
    // a fixed-capacity sparse wire: the first `cap` hits (index order) travel, the rest stay in
    // the error-feedback residual (or are dropped without EF) and are counted; with capacities
    // from the count exchange this cannot happen (cap = max over ranks of total)
    if (overflow != nullptr) atomicAdd(overflow, (unsigned long long)(S.total - S.cap));
    S.quota = S.cap > S.cnt_gt ? min(S.quota, S.cap - S.cnt_gt) : 0u;
    S.total = min(S.cnt_gt, S.cap) + S.quota;
  }
  st[li] = S;
}

__global__ __launch_bounds__(NT) void k_fill_tail(int2* __restrict__ pairs,
                                                  const int64_t* __restrict__ cap_off,
                                                  const int32_t* __restrict__ large_segs,
                                                  const SelState* __restrict__ st) {
  const int li = blockIdx.x;
  const int s = large_segs[li];
  const int64_t c0 = cap_off[s];
  const uint32_t cap = (uint32_t)(cap_off[s + 1] - c0);
  for (uint32_t p = st[li].total + threadIdx.x; p < cap; p += NT) pairs[c0 + p] = make_int2(SENT, 0);
}

// Order-preserving compaction. Thread owns EPT contiguous elements.
// FW (the fused chain): the workgroup of the segment's last task pads the unused pair slots
// (k_fill_tail) and zeroes the segment's radix histograms for the next call (so the chain needs
// no k_zero_words; the workspace starts zeroed). With prefix_from_cnt there is no k_scan either:
// the workgroup adds up the (gt, eq) counts of its segment's earlier tasks itself (`pre` is then
// the count array) — O(tasks²) loads per segment, so only when no segment has more than
// LW_FW_SCAN_MAX tasks (VGG-16's 103 M-weight layer has 12.6 k: it keeps k_scan).
template <int KM, int OUT, bool EF, bool FW = false>
__global__ __launch_bounds__(NT) void k_write(float* __restrict__ g, float* __restrict__ ef,
                                              const int64_t* __restrict__ seg_off,
                                              const int32_t* __restrict__ seg_n,
                                              const int32_t* __restrict__ large_segs,
                                              const int2* __restrict__ tasks,
                                              const SelState* __restrict__ st,
                                              const uint2* __restrict__ pre,
                                              const int64_t* __restrict__ cap_off,
                                              int2* __restrict__ pairs, float* __restrict__ vals,
                                              int32_t* __restrict__ idx_out, uint32_t gid_base,
                                              uint32_t step_arg, uint32_t s0, uint32_t s1, const uint32_t* __restrict__ stepp,
                                              float* __restrict__ mom,
                                              const int32_t* __restrict__ task_lo = nullptr,
                                              uint32_t* __restrict__ hist_all = nullptr,
                                              int prefix_from_cnt = 0) {
  // graph-captured steps read the step counter from device memory (csrc/lw_kernels.h)
  const uint32_t step = stepp != nullptr ? *stepp : step_arg;
  __shared__ uint32_t scr[NT / WAVE];
  // FW: kWriteSub workgroups per task, one per EPB / kWriteSub elements (a small bucket's write
  // then spreads over 4x the workgroups); `pre` / the count array are per sub-task
  constexpr int SUB = FW ? kWriteSub : 1;
  constexpr int EW = EPT / SUB;                 // elements per thread
  const int wi = (int)blockIdx.x;               // (sub-)task index
  const int2 t = tasks[wi / SUB];
  const int li = t.x, begin = t.y + (wi % SUB) * (EPB / SUB);
  const int s = large_segs[li];
  const int n = seg_n[s];
  const int64_t off = seg_off[s];
  const SelState S = st[li];
  uint2 bp;
  if (FW && prefix_from_cnt) {
    uint32_t sg = 0, se = 0;
    for (int q = task_lo[li] * SUB + (int)threadIdx.x; q < wi; q += NT) {
      const uint2 c = pre[q];
      sg += c.x;
      se += c.y;
    }
    block_excl_scan<NT>(sg, scr, bp.x);
    block_excl_scan<NT>(se, scr, bp.y);
  } else {
    bp = pre[wi];
  }
  const bool seg_last = FW && wi == task_lo[li + 1] * SUB - 1;
  if (seg_last) {
    uint32_t* hz = hist_all + (size_t)li * HIST_WORDS;
    for (int q = threadIdx.x; q < HIST_WORDS; q += NT) hz[q] = 0u;
  }
  // momentum factor masking (see k_small_select): only in segments not sent whole
  float* mp = (mom != nullptr && S.total < (uint32_t)n) ? mom + off : nullptr;
  const int64_t c0 = cap_off[s];
  float* gp = g + off;
  float* ep = EF ? ef + off : nullptr;
  const int i_base = begin + threadIdx.x * EW;
  const int end = min(begin + EPB / SUB, n);
  // RANDK never touched g in the histogram passes, so its EF add happens here.
  constexpr bool ADD_EF_HERE = EF && (KM == KM_RANDK);

  float v[EW];
  uint32_t key[EW];
  if (i_base + EW <= end) {
#pragma unroll
    for (int q = 0; q < EW / 4; ++q) {
      float4 x = *reinterpret_cast<const float4*>(gp + i_base + 4 * q);
      if (ADD_EF_HERE) {
        const float4 e = *reinterpret_cast<const float4*>(ep + i_base + 4 * q);
        x.x += e.x; x.y += e.y; x.z += e.z; x.w += e.w;
      }
      v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < EW; ++k) {
      const int i = i_base + k;
      float x = 0.f;
      if (i < end) { x = gp[i]; if (ADD_EF_HERE) x += ep[i]; }
      v[k] = x;
    }
  }
  if (KM == KM_RANDK) {
#pragma unroll
    for (int k = 0; k < EW; k += 4) {
      uint32_t q[4];
      randk_key4(i_base + k, gid_base + s, step, s0, s1, q);
      key[k] = q[0]; key[k + 1] = q[1]; key[k + 2] = q[2]; key[k + 3] = q[3];
    }
  } else {
#pragma unroll
    for (int k = 0; k < EW; ++k) key[k] = abs_key(v[k]);
  }
  uint32_t cg = 0, ce = 0;
#pragma unroll
  for (int k = 0; k < EW; ++k) {
    const bool ok = i_base + k < end;
    cg += ok && key[k] > S.tkey;
    ce += ok && key[k] == S.tkey;
  }
  uint32_t tot;
  const uint32_t p = block_excl_scan<NT>(cg | (ce << 16), scr, tot);
  uint32_t gb = bp.x + (p & 0xffffu), eb = bp.y + (p >> 16);
  float eo[EW];                                 // the residual left at each element
#pragma unroll
  for (int k = 0; k < EW; ++k) {
    const int i = i_base + k;
    eo[k] = v[k];
    if (i >= end) break;
    bool sel = false;
    uint32_t pos = 0;
    if (key[k] > S.tkey) { pos = gb + min(eb, S.quota); sel = pos < S.cap; ++gb; }
    else if (key[k] == S.tkey) { if (eb < S.quota) { pos = gb + eb; sel = pos < S.cap; } ++eb; }
    if (sel) {
      if (OUT == OUT_PAIRS) pairs[c0 + pos] = make_int2(i, __float_as_int(v[k]));
      else { vals[c0 + pos] = v[k]; idx_out[c0 + pos] = i; }
      if (mp != nullptr) mp[i] = 0.f;
      eo[k] = 0.f;
    }
  }
  // the residual as whole float4 stores (one per 4 elements, not one dword per lane each)
  if (EF) {
    if (i_base + EW <= end) {
#pragma unroll
      for (int q = 0; q < EW / 4; ++q)
        *reinterpret_cast<float4*>(ep + i_base + 4 * q) =
            make_float4(eo[4 * q], eo[4 * q + 1], eo[4 * q + 2], eo[4 * q + 3]);
    } else {
#pragma unroll
      for (int k = 0; k < EW; ++k)
        if (i_base + k < end) ep[i_base + k] = eo[k];
    }
  }
  // (k_fill_tail folded in: the workgroup of the segment's last task pads the unused pair slots;
  // no workgroup writes a slot at or past S.total)
  if (OUT == OUT_PAIRS && seg_last)
    for (uint32_t q = S.total + threadIdx.x; q < S.cap; q += NT) pairs[c0 + q] = make_int2(SENT, 0);
}

// ------------------------------------------------------------------------------------------
// Per-segment abs-max / sum-of-squares (two-level, fixed reduction order => deterministic)
// ------------------------------------------------------------------------------------------
template <bool EFADD>
__global__ __launch_bounds__(NT) void k_partial(float* __restrict__ g, const float* __restrict__ ef,
                                                const int64_t* __restrict__ seg_off,
                                                const int32_t* __restrict__ seg_n,
                                                const int32_t* __restrict__ large_segs,
                                                const int2* __restrict__ tasks,
                                                float2* __restrict__ partial) {
  __shared__ float scr[NT / WAVE];
  const int2 t = tasks[blockIdx.x];
  const int li = t.x, begin = t.y;
  const int s = large_segs[li];
  const int n = seg_n[s];
  const int64_t off = seg_off[s];
  float* gp = g + off;
  const float* ep = EFADD ? ef + off : nullptr;
  const int end = min(begin + EPB, n);
  float mx = 0.f, ss = 0.f;
  for (int j = 0; j < EPB / (NT * 4); ++j) {
    const int i0 = begin + j * NT * 4 + threadIdx.x * 4;
    if (i0 >= end) break;
    float4 v;
    if (i0 + 3 < end) {
      v = *reinterpret_cast<const float4*>(gp + i0);
      if (EFADD) {
        const float4 e = *reinterpret_cast<const float4*>(ep + i0);
        v.x += e.x; v.y += e.y; v.z += e.z; v.w += e.w;
        *reinterpret_cast<float4*>(gp + i0) = v;
      }
    } else {
      float t4[4] = {0.f, 0.f, 0.f, 0.f};
      for (int q = 0; q < 4; ++q)
        if (i0 + q < end) {
          float x = gp[i0 + q];
          if (EFADD) { x += ep[i0 + q]; gp[i0 + q] = x; }
          t4[q] = x;
        }
      v = make_float4(t4[0], t4[1], t4[2], t4[3]);
    }
    mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  mx = block_max<NT>(mx, scr);
  ss = block_sum<NT>(ss, scr);
  if (threadIdx.x == 0) partial[blockIdx.x] = make_float2(mx, ss);
}

// out[li] = max (what=0) or sqrt(sum sq) (what=1)
__global__ __launch_bounds__(NT) void k_finalize(const float2* __restrict__ partial,
                                                 const int32_t* __restrict__ task_lo,
                                                 float* __restrict__ out, int what) {
  __shared__ float scr[NT / WAVE];
  const int li = blockIdx.x;
  const int lo = task_lo[li], hi = task_lo[li + 1];
  float mx = 0.f, ss = 0.f;
  for (int i = lo + threadIdx.x; i < hi; i += NT) {
    const float2 p = partial[i];
    mx = fmaxf(mx, p.x);
    ss += p.y;
  }
  mx = block_max<NT>(mx, scr);
  ss = block_sum<NT>(ss, scr);
  if (threadIdx.x == 0) out[li] = what == 0 ? mx : sqrtf(ss);
}

// ------------------------------------------------------------------------------------------
// Quantisers. Payload (int32 words, per rank): [nseg header floats][records], segment li's
// group records at hdr + rec_off[li]*R words (a group = 32 consecutive elements).
//   Q_TERN : 2-bit codes {0, +1, -1}: R = 2
//   Q_QS8  : signed int8 level, qstates <= 127: R = 8
//   Q_QS9  : uint8 level + sign bitmap, qstates <= 255: 8 level words at rec*8 and the sign
//            word at the segment's sign block (levels block: G*8 words, then G sign words)
//   Q_QS16 : signed int16 level, qstates <= 32767: R = 16
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void rng32(float u[EPT], uint32_t i_base, uint32_t gid, uint32_t step,
                                      uint32_t tag, uint32_t s0, uint32_t s1) {
#pragma unroll
  for (int k = 0; k < EPT; k += 4) {
    const u4 r = philox4x32_10(u4{(i_base + k) >> 2, gid, step, tag}, s0, s1);
    u[k] = u01(r.x); u[k + 1] = u01(r.y); u[k + 2] = u01(r.z); u[k + 3] = u01(r.w);
  }
}

template <int Q, bool EF>
__global__ __launch_bounds__(NT) void k_quant(
    const float* __restrict__ g, float* __restrict__ ef, const int64_t* __restrict__ seg_off,
    const int32_t* __restrict__ seg_n, const int32_t* __restrict__ large_segs,
    const int2* __restrict__ tasks, const int64_t* __restrict__ rec_off,
    const float* __restrict__ scale, uint32_t* __restrict__ payload, int nseg, int qstates,
    uint32_t gid_base, uint32_t step_arg, uint32_t tag, uint32_t s0, uint32_t s1,
    const uint32_t* __restrict__ stepp) {
  const uint32_t step = stepp != nullptr ? *stepp : step_arg;
  const int2 t = tasks[blockIdx.x];
  const int li = t.x, begin = t.y;
  const int s = large_segs[li];
  const int n = seg_n[s];
  const int64_t off = seg_off[s];
  const float sc = scale[li];
  if (t.y == 0 && threadIdx.x == 0) payload[li] = __float_as_uint(sc);
  const int i_base = begin + threadIdx.x * EPT;
  if (i_base >= n) return;
  const int end = min(begin + EPB, n);
  const float* gp = g + off;
  float* ep = EF ? ef + off : nullptr;
  float v[EPT];
  if (i_base + EPT <= end) {
#pragma unroll
    for (int q = 0; q < EPT / 4; ++q) {
      const float4 x = *reinterpret_cast<const float4*>(gp + i_base + 4 * q);
      v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < EPT; ++k) v[k] = (i_base + k < end) ? gp[i_base + k] : 0.f;
  }
  float u[EPT];
  rng32(u, (uint32_t)i_base, gid_base + s, step, tag, s0, s1);
  const int64_t grp = rec_off[li] + i_base / EPT;   // group index within payload records
  uint32_t* rec = payload + hdr_words(nseg);
  float dq[EPT];
  if (Q == Q_TERN) {
    uint32_t w0 = 0, w1 = 0;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      uint32_t c = 0;
      if (sc > 0.f) {
        const float prob = fabsf(v[k]) / sc;
        if (u[k] < prob) c = v[k] > 0.f ? 1u : (v[k] < 0.f ? 2u : 0u);
      }
      dq[k] = c == 1u ? sc : (c == 2u ? -sc : 0.f);
      if (k < 16) w0 |= c << (2 * k); else w1 |= c << (2 * (k - 16));
    }
    *reinterpret_cast<uint2*>(rec + grp * 2) = make_uint2(w0, w1);
  } else {
    const float qs = (float)qstates;
    int lv[EPT];
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      int l = 0;
      if (sc > 0.f) {
        l = (int)floorf(fabsf(v[k]) / sc * qs + u[k]);
        l = min(l, qstates);
      }
      const float sg = v[k] > 0.f ? 1.f : (v[k] < 0.f ? -1.f : 0.f);
      dq[k] = sg * sc * ((float)l / qs);
      lv[k] = v[k] < 0.f ? -l : l;
    }
    if (Q == Q_QS8) {
      uint32_t w[8];
#pragma unroll
      for (int q = 0; q < 8; ++q)
        w[q] = (uint32_t)(lv[4 * q] & 0xff) | ((uint32_t)(lv[4 * q + 1] & 0xff) << 8) |
               ((uint32_t)(lv[4 * q + 2] & 0xff) << 16) | ((uint32_t)(lv[4 * q + 3] & 0xff) << 24);
      uint4* o = reinterpret_cast<uint4*>(rec + grp * 8);
      o[0] = make_uint4(w[0], w[1], w[2], w[3]);
      o[1] = make_uint4(w[4], w[5], w[6], w[7]);
    } else if (Q == Q_QS9) {
      const int64_t Gtot = rec_off[nseg];     // all level words first, then all sign words
      uint32_t w[8], sgn = 0;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        w[q] = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int l = lv[4 * q + r];
          w[q] |= (uint32_t)(l < 0 ? -l : l) << (8 * r);
          sgn |= (l < 0 ? 1u : 0u) << (4 * q + r);
        }
      }
      uint4* o = reinterpret_cast<uint4*>(rec + grp * 8);
      o[0] = make_uint4(w[0], w[1], w[2], w[3]);
      o[1] = make_uint4(w[4], w[5], w[6], w[7]);
      rec[Gtot * 8 + grp] = sgn;
    } else {  // Q_QS16
      uint32_t w[16];
#pragma unroll
      for (int q = 0; q < 16; ++q)
        w[q] = (uint32_t)(lv[2 * q] & 0xffff) | ((uint32_t)(lv[2 * q + 1] & 0xffff) << 16);
      uint4* o = reinterpret_cast<uint4*>(rec + grp * 16);
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
    }
  }
  if (EF) {
#pragma unroll
    for (int k = 0; k < EPT; ++k)
      if (i_base + k < end) ep[i_base + k] = v[k] - dq[k];
  }
}

// Dequantise every rank's payload for this thread's 32-element group, summing in rank order, then
// divide by the world size (core.py:221-223 `compress_grad /= float(world_size)`).
template <int Q>
__global__ __launch_bounds__(NT) void k_dequant(const uint32_t* __restrict__ gathered,
                                                int64_t words_per_rank, int ws,
                                                float* __restrict__ g,
                                                const int64_t* __restrict__ seg_off,
                                                const int32_t* __restrict__ seg_n,
                                                const int32_t* __restrict__ large_segs,
                                                const int2* __restrict__ tasks,
                                                const int64_t* __restrict__ rec_off, int nseg,
                                                int qstates) {
  const int2 t = tasks[blockIdx.x];
  const int li = t.x, begin = t.y;
  const int s = large_segs[li];
  const int n = seg_n[s];
  const int64_t off = seg_off[s];
  const int i_base = begin + threadIdx.x * EPT;
  if (i_base >= n) return;
  const int end = min(begin + EPB, n);
  const int64_t grp = rec_off[li] + i_base / EPT;
  const int64_t Gtot = rec_off[nseg];
  float acc[EPT];
#pragma unroll
  for (int k = 0; k < EPT; ++k) acc[k] = 0.f;
  for (int r = 0; r < ws; ++r) {
    const uint32_t* P = gathered + (int64_t)r * words_per_rank;
    const float sc = __uint_as_float(P[li]);
    const uint32_t* rec = P + hdr_words(nseg);
    if (Q == Q_TERN) {
      const uint2 w = *reinterpret_cast<const uint2*>(rec + grp * 2);
#pragma unroll
      for (int k = 0; k < EPT; ++k) {
        const uint32_t c = ((k < 16 ? w.x : w.y) >> (2 * (k & 15))) & 3u;
        acc[k] += c == 1u ? sc : (c == 2u ? -sc : 0.f);
      }
    } else if (Q == Q_QS8) {
      const uint4* o = reinterpret_cast<const uint4*>(rec + grp * 8);
      const uint4 a = o[0], b = o[1];
      const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
      for (int k = 0; k < EPT; ++k) {
        const int l = (int)(int8_t)((w[k >> 2] >> (8 * (k & 3))) & 0xff);
        const float sg = l > 0 ? 1.f : (l < 0 ? -1.f : 0.f);
        acc[k] += sg * sc * ((float)(l < 0 ? -l : l) / (float)qstates);
      }
    } else if (Q == Q_QS9) {
      const uint4* o = reinterpret_cast<const uint4*>(rec + grp * 8);
      const uint4 a = o[0], b = o[1];
      const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      const uint32_t sgn = rec[Gtot * 8 + grp];
#pragma unroll
      for (int k = 0; k < EPT; ++k) {
        const int l = (int)((w[k >> 2] >> (8 * (k & 3))) & 0xff);
        const float sg = l == 0 ? 0.f : (((sgn >> k) & 1u) ? -1.f : 1.f);
        acc[k] += sg * sc * ((float)l / (float)qstates);
      }
    } else {
      const uint4* o = reinterpret_cast<const uint4*>(rec + grp * 16);
      uint32_t w[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 x = o[q];
        w[4 * q] = x.x; w[4 * q + 1] = x.y; w[4 * q + 2] = x.z; w[4 * q + 3] = x.w;
      }
#pragma unroll
      for (int k = 0; k < EPT; ++k) {
        const int l = (int)(int16_t)((w[k >> 1] >> (16 * (k & 1))) & 0xffff);
        const float sg = l > 0 ? 1.f : (l < 0 ? -1.f : 0.f);
        acc[k] += sg * sc * ((float)(l < 0 ? -l : l) / (float)qstates);
      }
    }
  }
  float* gp = g + off;
  const float fws = (float)ws;
  if (i_base + EPT <= end) {
#pragma unroll
    for (int q = 0; q < EPT / 4; ++q)
      *reinterpret_cast<float4*>(gp + i_base + 4 * q) =
          make_float4(acc[4 * q] / fws, acc[4 * q + 1] / fws, acc[4 * q + 2] / fws,
                      acc[4 * q + 3] / fws);
  } else {
    for (int k = 0; k < EPT; ++k)
      if (i_base + k < end) gp[i_base + k] = acc[k] / fws;
  }
}

// ------------------------------------------------------------------------------------------
// Unpack of all-gathered (index, value) pairs: deterministic rank-ordered sum, / world_size.
// ------------------------------------------------------------------------------------------
// First position in a[0..len) whose .x >= x (a sorted by .x): 64-ary search by one wave.
__device__ __forceinline__ int wave_lower_bound(const int2* __restrict__ a, int len, int x) {
  const int lane = threadIdx.x & (WAVE - 1);
  int lo = 0, hi = len;
  while (hi - lo > WAVE) {
    const int step = (hi - lo + WAVE - 1) / WAVE;
    const int p = lo + lane * step;
    const bool pred = (p < hi) && (a[p].x < x);
    const int c = __popcll(__ballot(pred));
    if (c == 0) { hi = lo; }
    else {
      const int plast = lo + (c - 1) * step;
      const int pnext = lo + c * step;
      lo = plast + 1;
      hi = min(pnext, hi);
    }
  }
  const int p = lo + lane;
  const bool pred = (p < hi) && (a[p].x < x);
  return lo + __popcll(__ballot(pred));
}

constexpr int UCH = kUnpackChunk;   // 4096 elements per workgroup

// Rank-ordered LDS accumulation of every rank's pairs that fall in the 4096-element chunk
// [cb, ce) of segment s (deterministic: ranks in order, a rank's pairs in index order).
__device__ __forceinline__ void unpack_acc(const int2* __restrict__ gathered, int64_t cap_total,
                                           int ws, const int64_t* __restrict__ cap_off, int s,
                                           int cb, int ce, float* acc, int* lo_s, int* hi_s) {
  const int64_t c0 = cap_off[s];
  const int cap = (int)(cap_off[s + 1] - c0);
  for (int j = threadIdx.x; j < UCH; j += NT) acc[j] = 0.f;
  const int w = threadIdx.x / WAVE;
  for (int r = w; r < ws; r += NT / WAVE) {
    const int2* a = gathered + (int64_t)r * cap_total + c0;
    const int l = wave_lower_bound(a, cap, cb);
    const int h = wave_lower_bound(a, cap, ce);
    if ((threadIdx.x & (WAVE - 1)) == 0) { lo_s[r] = l; hi_s[r] = h; }
  }
  __syncthreads();
  for (int r = 0; r < ws; ++r) {
    const int2* a = gathered + (int64_t)r * cap_total + c0;
    for (int j = lo_s[r] + threadIdx.x; j < hi_s[r]; j += NT) {
      const int2 p = a[j];
      acc[p.x - cb] += __int_as_float(p.y);
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(NT) void k_unpack_pairs(const int2* __restrict__ gathered,
                                                     int64_t cap_total, int ws,
                                                     float* __restrict__ g,
                                                     const int64_t* __restrict__ seg_off,
                                                     const int32_t* __restrict__ seg_n,
                                                     const int64_t* __restrict__ cap_off,
                                                     const int2* __restrict__ utasks) {
  __shared__ float acc[UCH];
  __shared__ int lo_s[kMaxWorld], hi_s[kMaxWorld];
  const int2 t = utasks[blockIdx.x];
  const int s = t.x, cb = t.y;
  const int ce = min(cb + UCH, seg_n[s]);
  unpack_acc(gathered, cap_total, ws, cap_off, s, cb, ce, acc, lo_s, hi_s);
  float* gp = g + seg_off[s] + cb;
  const float fws = (float)ws;
  const int len = ce - cb;
  if (len == UCH) {
    for (int j = threadIdx.x * 4; j < UCH; j += NT * 4)
      *reinterpret_cast<float4*>(gp + j) =
          make_float4(acc[j] / fws, acc[j + 1] / fws, acc[j + 2] / fws, acc[j + 3] / fws);
  } else {
    for (int j = threadIdx.x; j < len; j += NT) gp[j] = acc[j] / fws;
  }
}

// Decode and optimizer step in one pass (Top-K buckets; parallel/engine.py set_fused_sgd): the
// chunk's averaged gradient goes from LDS straight into the SGD update of the same elements
// (sgd_elem, as k_sgd) — the dense gradient is neither written by the decode nor read back by the
// optimizer. A task {codec segment, chunk begin, chunk end, parameter} never crosses a parameter
// (entire-model buckets: chunks are cut at the arena's segment boundaries), so its weight decay
// is a.seg_wd[parameter]. `a` points at the bucket: a.p / a.buf / a.pb at its first element,
// a.seg_wd at its first parameter.
template <bool MOM, bool NEST, bool FIRST>
__global__ __launch_bounds__(NT) void k_unpack_sgd(const int2* __restrict__ gathered,
                                                   int64_t cap_total, int ws,
                                                   const int64_t* __restrict__ seg_off,
                                                   const int64_t* __restrict__ cap_off,
                                                   const int4* __restrict__ ftasks,
                                                   const SgdArgs a) {
  __shared__ float acc[UCH];
  __shared__ int lo_s[kMaxWorld], hi_s[kMaxWorld];
  const int4 t = ftasks[blockIdx.x];
  const int s = t.x, cb = t.y, ce = t.z;
  unpack_acc(gathered, cap_total, ws, cap_off, s, cb, ce, acc, lo_s, hi_s);
  float lr = a.lr, grad_scale = a.grad_scale;
  if (a.hyper != nullptr) {
    lr = a.hyper[0];
    grad_scale = a.hyper[1];
  }
  const float wd = a.seg_wd[t.w];
  const int64_t off = seg_off[s] + cb;
  float* pp = a.p + off;
  float* bp = a.buf + off;
  uint16_t* hp = a.pb != nullptr ? a.pb + off : nullptr;
  const float fws = (float)ws;
  const int len = ce - cb;
  if (len == UCH && (off & 3) == 0) {
    for (int j = threadIdx.x * 4; j < UCH; j += NT * 4) {
      const float4 x4 = *reinterpret_cast<const float4*>(pp + j);
      float x[4] = {x4.x, x4.y, x4.z, x4.w};
      float b[4] = {0.f, 0.f, 0.f, 0.f};
      if (MOM && !FIRST) {
        const float4 b4 = *reinterpret_cast<const float4*>(bp + j);
        b[0] = b4.x; b[1] = b4.y; b[2] = b4.z; b[3] = b4.w;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
        x[k] = sgd_elem<MOM, NEST, FIRST>(x[k], acc[j + k] / fws, b[k], lr, wd, a.momentum,
                                          a.dampening, grad_scale);
      *reinterpret_cast<float4*>(pp + j) = make_float4(x[0], x[1], x[2], x[3]);
      if (MOM) *reinterpret_cast<float4*>(bp + j) = make_float4(b[0], b[1], b[2], b[3]);
      if (hp != nullptr)
        *reinterpret_cast<uint2*>(hp + j) =
            make_uint2((uint32_t)f2h(x[0]) | ((uint32_t)f2h(x[1]) << 16),
                       (uint32_t)f2h(x[2]) | ((uint32_t)f2h(x[3]) << 16));
    }
  } else {
    for (int j = threadIdx.x; j < len; j += NT) {
      float b = MOM && !FIRST ? bp[j] : 0.f;
      const float x = sgd_elem<MOM, NEST, FIRST>(pp[j], acc[j] / fws, b, lr, wd, a.momentum,
                                                 a.dampening, grad_scale);
      pp[j] = x;
      if (MOM) bp[j] = b;
      if (hp != nullptr) hp[j] = f2h(x);
    }
  }
}

// Index-free Random-K: every rank selected the same indices; values were all-reduced (summed).
__global__ __launch_bounds__(NT) void k_unpack_validx(const float* __restrict__ vals,
                                                      const int32_t* __restrict__ idx,
                                                      const int32_t* __restrict__ slot_seg,
                                                      int64_t nslots, int ws,
                                                      float* __restrict__ g,
                                                      const int64_t* __restrict__ seg_off) {
  const int64_t j = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (j >= nslots) return;
  const int s = slot_seg[j];
  g[seg_off[s] + idx[j]] = vals[j] / (float)ws;
}

// ------------------------------------------------------------------------------------------
// Host launchers
// ------------------------------------------------------------------------------------------
#define LW_LAUNCH(kern, grid, stream, ...) \
  hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), 0, stream, __VA_ARGS__)

// Histogram reset as a kernel of our own, NOT hipMemsetAsync: inside a replayed HIP graph the
// runtime's memset node (the __amd_rocclr_fillBufferAligned blit) was seen to fill this buffer with
// a non-zero periodic pattern after a few replays (bin sums 2:1:1 across the 2048/1024/1024-bin
// pass regions, i.e. a repeated garbage word pattern, on top of which k_hist added its counts),
// which made the radix select pick a threshold no key reached: nothing was sent and the error
// feedback kept the whole gradient (scripts/probes/replay_bisect.py,
// profiles/r3_graph_divergence_root_cause.md). Stream-ordered kernels only, here and everywhere
// else on the captured path.
__global__ __launch_bounds__(NT) void k_zero_words(uint32_t* __restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT)
    p[i] = 0u;
}

// tasks per histogram / count workgroup: LW_HIST_TPB on large launches, 1 on mid-sized ones and,
// below LW_HIST_SPLIT_MAX tasks, -kWriteSub: each task split over kWriteSub workgroups (k_hist,
// k_count_sel). (Every workgroup zeroes and flushes a whole LDS histogram per segment: splitting a
// ResNet-50 bucket's ~1.2 k tasks 4 ways cost 0.3 ms a step; AlexNet's one 281-task bucket gains.)
#ifndef LW_HIST_SPLIT_MAX
#define LW_HIST_SPLIT_MAX 512
#endif
static int hist_tpb(int ntasks) {
  return ntasks >= LW_HIST_TPB_MIN ? LW_HIST_TPB : (ntasks < LW_HIST_SPLIT_MAX ? -kWriteSub : 1);
}
static int hist_blocks(int ntasks) {
  const int t = hist_tpb(ntasks);
  return t > 0 ? (ntasks + t - 1) / t : ntasks * -t;
}
// Pass 0 of a split launch: LW_HIST0_SPLIT workgroups per task (1, 2 or 4). Not split: pass 0
// counts every key, so each of its workgroups merges a dense 2048-bin histogram into the
// segment's one with global atomics — executed at the memory side, where adds to one word
// serialise — and 4x the workgroups meant 4x those merges: AlexNet's 276-task entire-model
// bucket 25 -> 14 µs (scripts/probes/select_probe.hip, profiles/r5/select_probe.jsonl).
#ifndef LW_HIST0_SPLIT
#define LW_HIST0_SPLIT 1
#endif
static int hist0_tpb(int ntasks) {
  const int t = hist_tpb(ntasks);
  return t > 0 ? t : -LW_HIST0_SPLIT;
}
static int hist0_blocks(int ntasks) {
  const int t = hist0_tpb(ntasks);
  return t > 0 ? (ntasks + t - 1) / t : ntasks * -t;
}
// Pass 0 of a launch whose longest segment has LW_HIST0_BIG_MIN tasks or more: 1024-thread
// workgroups of several tasks each (shorter segments: the 256-thread grid above). The histogram
// merges execute one per word at the memory side, so their time grows with how many workgroups
// add into one segment's hot bins, not with the workgroup size. Tasks per workgroup = the longest
// segment's tasks / 64 (2..16): about 64 merges per hot bin while a layer-wise bucket keeps
// hundreds of workgroups for its bandwidth. Same keys per thread, same waves per launch.
// AlexNet's 276-task entire-model bucket: pass 0 13.8 -> 10.7 µs on its real gradient; 9 M
// elements 39 -> 29 µs (profiles/r5/select_probe_hist0_big.jsonl).
#ifndef LW_HIST0_BIG_MIN
#define LW_HIST0_BIG_MIN 128
#endif
constexpr int TB0 = 1024;
static int hist0_big_tpb(int max_seg_tasks) {
  if (max_seg_tasks < LW_HIST0_BIG_MIN) return 0;
  return std::min(16, std::max(2, max_seg_tasks / 64));
}

template <int KM, bool EFADD, bool MC>
static void launch_hist0(const SelectArgs& a, const int2* tk, int nt, hipStream_t st) {
  if (const int t = hist0_big_tpb(a.max_seg_tasks)) {
    hipLaunchKernelGGL((k_hist<KM, 0, EFADD, false, MC, TB0>), dim3((nt + t - 1) / t), dim3(TB0),
                       0, st, a.g, a.ef, a.seg_off, a.seg_n, a.large_segs, tk, nt, t, a.st_large,
                       a.hist, a.gid_base, a.step, a.seed0, a.seed1, a.step_ptr,
                       (const int32_t*)nullptr, (const int32_t*)nullptr, a.mcx);
  } else {
    LW_LAUNCH((k_hist<KM, 0, EFADD, false, MC>), hist0_blocks(nt), st, a.g, a.ef, a.seg_off,
              a.seg_n, a.large_segs, tk, nt, hist0_tpb(nt), a.st_large, a.hist, a.gid_base,
              a.step, a.seed0, a.seed1, a.step_ptr, (const int32_t*)nullptr,
              (const int32_t*)nullptr, a.mcx);
  }
}

template <int KM, int OUT, bool EF, bool MC = false>
static void select_compress_t(const SelectArgs& a, bool staged, hipStream_t st) {
  if (a.n_small > 0)
    LW_LAUNCH((k_small_select<KM, OUT, EF, MC>), a.n_small, st, a.g, a.ef, a.seg_off, a.seg_n,
              a.keep, a.cap_off, a.small_segs, a.pairs, a.vals, a.idx_out, a.st_small,
              a.gid_base, a.step, a.seed0, a.seed1, a.step_ptr, a.overflow, a.mom, a.mcx);
  if (a.n_large == 0) return;
  if (!staged) {      // (staged: select_stage already zeroed the histograms and ran pass 0)
    if (!LW_FUSED_SELECT) {    // (fused: the previous call's k_write left them zeroed)
      const int64_t words = (int64_t)HIST_WORDS * a.n_large;
      const int64_t nb = (words + NT - 1) / NT;
      LW_LAUNCH(k_zero_words, (int)(nb < 1024 ? nb : 1024), st, a.hist, words);
    }
    launch_hist0<KM, EF && KM == KM_TOPK, MC>(a, a.tasks, a.n_tasks, st);
  }
  if (LW_FUSED_SELECT) {
    // 4-5 launches instead of 11: the digit selections ride in the next pass's workgroups; the
    // payload tail padding, the histogram reset and (short segments) the count scan in k_write
    // (passes 1 / 2 stay on the 256-thread grid: on pass 0's multi-task 1024-thread grid they
    // measured slower — AlexNet pass 2 5.6 -> 8.8 µs, VGG-16 113.2 k -> 111.2 k img/s)
    LW_LAUNCH((k_hist<KM, 1, false, true>), hist_blocks(a.n_tasks), st, a.g, a.ef, a.seg_off,
              a.seg_n, a.large_segs, a.tasks, a.n_tasks, hist_tpb(a.n_tasks), a.st_large, a.hist, a.gid_base, a.step,
              a.seed0, a.seed1, a.step_ptr, a.keep, a.task_lo);
    LW_LAUNCH((k_hist<KM, 2, false, true>), hist_blocks(a.n_tasks), st, a.g, a.ef, a.seg_off,
              a.seg_n, a.large_segs, a.tasks, a.n_tasks, hist_tpb(a.n_tasks), a.st_large, a.hist, a.gid_base, a.step,
              a.seed0, a.seed1, a.step_ptr, a.keep, a.task_lo);
    LW_LAUNCH((k_count_sel<KM>), hist_blocks(a.n_tasks), st, a.g, a.seg_off, a.seg_n,
              a.large_segs, a.tasks, a.n_tasks, hist_tpb(a.n_tasks), a.task_lo, a.st_large, a.hist,
              a.keep, a.cap_off,
              a.overflow, a.cnt, a.gid_base, a.step, a.seed0, a.seed1, a.step_ptr);
    const bool own_prefix = a.max_seg_tasks > 0 && a.max_seg_tasks <= LW_FW_SCAN_MAX;
    if (!own_prefix)
      LW_LAUNCH((k_scan<KM>), a.n_large, st, a.cnt, a.pre, a.task_lo, a.st_large,
                (int32_t*)nullptr, kWriteSub);
    LW_LAUNCH((k_write<KM, OUT, EF, true>), a.n_tasks * kWriteSub, st, a.g, a.ef, a.seg_off,
              a.seg_n,
              a.large_segs, a.tasks, a.st_large, own_prefix ? a.cnt : a.pre, a.cap_off, a.pairs,
              a.vals, a.idx_out, a.gid_base, a.step, a.seed0, a.seed1, a.step_ptr, a.mom,
              a.task_lo, a.hist, own_prefix ? 1 : 0);
    return;
  }
  LW_LAUNCH((k_select<KM, 0>), a.n_large, st, a.hist, a.st_large, a.large_segs, a.keep, a.cap_off,
            a.overflow);
  LW_LAUNCH((k_hist<KM, 1, false>), hist_blocks(a.n_tasks), st, a.g, a.ef, a.seg_off, a.seg_n,
            a.large_segs, a.tasks, a.n_tasks, hist_tpb(a.n_tasks), a.st_large, a.hist, a.gid_base, a.step, a.seed0, a.seed1, a.step_ptr);
  LW_LAUNCH((k_select<KM, 1>), a.n_large, st, a.hist, a.st_large, a.large_segs, a.keep, a.cap_off,
            a.overflow);
  LW_LAUNCH((k_hist<KM, 2, false>), hist_blocks(a.n_tasks), st, a.g, a.ef, a.seg_off, a.seg_n,
            a.large_segs, a.tasks, a.n_tasks, hist_tpb(a.n_tasks), a.st_large, a.hist, a.gid_base, a.step, a.seed0, a.seed1, a.step_ptr);
  LW_LAUNCH((k_select<KM, 2>), a.n_large, st, a.hist, a.st_large, a.large_segs, a.keep, a.cap_off,
            a.overflow);
  LW_LAUNCH((k_count<KM, false>), a.n_tasks, st, a.g, a.ef, a.seg_off, a.seg_n, a.large_segs,
            a.tasks, a.st_large, a.cnt, a.gid_base, a.step, a.seed0, a.seed1, a.step_ptr);
  LW_LAUNCH((k_scan<KM>), a.n_large, st, a.cnt, a.pre, a.task_lo, a.st_large, (int32_t*)nullptr);
  if (OUT == OUT_PAIRS)
    LW_LAUNCH(k_fill_tail, a.n_large, st, a.pairs, a.cap_off, a.large_segs, a.st_large);
  LW_LAUNCH((k_write<KM, OUT, EF>), a.n_tasks, st, a.g, a.ef, a.seg_off, a.seg_n, a.large_segs,
            a.tasks, a.st_large, a.pre, a.cap_off, a.pairs, a.vals, a.idx_out, a.gid_base, a.step,
            a.seed0, a.seed1, a.step_ptr, a.mom);
}

void select_compress(const SelectArgs& a, int km, int out, bool ef, hipStream_t st, bool staged) {
  if (a.mcx.u != nullptr) {      // fused momentum correction: Top-K pairs, unstaged
    if (km != KM_TOPK || out != OUT_PAIRS || staged) return;   // (rejected by the binding)
    ef ? select_compress_t<KM_TOPK, OUT_PAIRS, true, true>(a, false, st)
       : select_compress_t<KM_TOPK, OUT_PAIRS, false, true>(a, false, st);
    return;
  }
  if (km == KM_TOPK && out == OUT_PAIRS) {
    ef ? select_compress_t<KM_TOPK, OUT_PAIRS, true>(a, staged, st)
       : select_compress_t<KM_TOPK, OUT_PAIRS, false>(a, staged, st);
  } else if (km == KM_RANDK && out == OUT_VALIDX) {
    ef ? select_compress_t<KM_RANDK, OUT_VALIDX, true>(a, staged, st)
       : select_compress_t<KM_RANDK, OUT_VALIDX, false>(a, staged, st);
  } else if (km == KM_RANDK && out == OUT_PAIRS) {
    ef ? select_compress_t<KM_RANDK, OUT_PAIRS, true>(a, staged, st)
       : select_compress_t<KM_RANDK, OUT_PAIRS, false>(a, staged, st);
  } else {
    ef ? select_compress_t<KM_TOPK, OUT_VALIDX, true>(a, staged, st)
       : select_compress_t<KM_TOPK, OUT_VALIDX, false>(a, staged, st);
  }
}

// Entire-model staging (parallel/engine.py): the one segment's first pass — the radix pass-0
// histogram with the error-feedback fold g' = g + e (Top-K), or the histogram of the Philox keys
// (Random-K) — over tasks [t_lo, t_hi), launched while backward still runs, as the arena slice
// those tasks cover completes. The counts are integers added atomically, so any split of the tasks
// gives the histogram of one launch; select_compress(staged) then runs the rest of the chain.
void select_stage(const SelectArgs& a, int km, bool ef, int t_lo, int t_hi, bool zero,
                  hipStream_t st) {
  if (zero) {
    const int64_t words = (int64_t)HIST_WORDS * a.n_large;
    const int64_t nb = (words + NT - 1) / NT;
    LW_LAUNCH(k_zero_words, (int)(nb < 1024 ? nb : 1024), st, a.hist, words);
  }
  if (t_hi <= t_lo) return;
  const int2* tk = a.tasks + t_lo;
  if (km == KM_TOPK) {
    if (ef) launch_hist0<KM_TOPK, true, false>(a, tk, t_hi - t_lo, st);
    else launch_hist0<KM_TOPK, false, false>(a, tk, t_hi - t_lo, st);
  } else {
    launch_hist0<KM_RANDK, false, false>(a, tk, t_hi - t_lo, st);
  }
}

void thresh_count(const SelectArgs& a, float V, int adaptive, bool ef, float* segmax,
                  float2* partial, int32_t* count_out, hipStream_t st) {
  if (adaptive) {
    if (ef) LW_LAUNCH((k_partial<true>), a.n_tasks, st, a.g, a.ef, a.seg_off, a.seg_n, a.large_segs, a.tasks, partial);
    else LW_LAUNCH((k_partial<false>), a.n_tasks, st, a.g, a.ef, a.seg_off, a.seg_n, a.large_segs, a.tasks, partial);
    LW_LAUNCH(k_finalize, a.n_large, st, partial, a.task_lo, segmax, 0);
  }
  hipLaunchKernelGGL(k_thresh_state, dim3((a.n_large + NT - 1) / NT), dim3(NT), 0, st, a.st_large,
                     (const float*)segmax, a.n_large, V, adaptive);
  if (ef && !adaptive)
    LW_LAUNCH((k_count<KM_THRESH, true>), a.n_tasks, st, a.g, a.ef, a.seg_off, a.seg_n,
              a.large_segs, a.tasks, a.st_large, a.cnt, 0u,  0u, 0u, 0u, (const uint32_t*)nullptr);
  else
    LW_LAUNCH((k_count<KM_THRESH, false>), a.n_tasks, st, a.g, a.ef, a.seg_off, a.seg_n,
              a.large_segs, a.tasks, a.st_large, a.cnt, 0u,  0u, 0u, 0u, (const uint32_t*)nullptr);
  LW_LAUNCH((k_scan<KM_THRESH>), a.n_large, st, a.cnt, a.pre, a.task_lo, a.st_large, count_out);
}

void thresh_dense(const SelectArgs& a, float V, int adaptive, bool ef, float* segmax,
                  float2* partial, hipStream_t st) {
  if (adaptive) {
    if (ef) LW_LAUNCH((k_partial<true>), a.n_tasks, st, a.g, a.ef, a.seg_off, a.seg_n, a.large_segs, a.tasks, partial);
    else LW_LAUNCH((k_partial<false>), a.n_tasks, st, a.g, a.ef, a.seg_off, a.seg_n, a.large_segs, a.tasks, partial);
    LW_LAUNCH(k_finalize, a.n_large, st, partial, a.task_lo, segmax, 0);
  }
  hipLaunchKernelGGL(k_thresh_state, dim3((a.n_large + NT - 1) / NT), dim3(NT), 0, st, a.st_large,
                     (const float*)segmax, a.n_large, V, adaptive);
  if (ef && !adaptive)
    LW_LAUNCH((k_thresh_dense<true, true>), a.n_tasks, st, a.g, a.ef, a.seg_off, a.seg_n,
              a.large_segs, a.tasks, a.st_large);
  else if (ef)   // k_partial<true> already folded the residual into g
    LW_LAUNCH((k_thresh_dense<false, true>), a.n_tasks, st, a.g, a.ef, a.seg_off, a.seg_n,
              a.large_segs, a.tasks, a.st_large);
  else
    LW_LAUNCH((k_thresh_dense<false, false>), a.n_tasks, st, a.g, a.ef, a.seg_off, a.seg_n,
              a.large_segs, a.tasks, a.st_large);
}

void thresh_write(const SelectArgs& a, bool ef, hipStream_t st) {
  hipLaunchKernelGGL(k_set_caps, dim3((a.n_large + NT - 1) / NT), dim3(NT), 0, st, a.st_large,
                     a.cap_off, a.large_segs, a.n_large, a.overflow);
  LW_LAUNCH(k_fill_tail, a.n_large, st, a.pairs, a.cap_off, a.large_segs, a.st_large);
  if (ef)
    LW_LAUNCH((k_write<KM_THRESH, OUT_PAIRS, true>), a.n_tasks, st, a.g, a.ef, a.seg_off, a.seg_n,
              a.large_segs, a.tasks, a.st_large, a.pre, a.cap_off, a.pairs, a.vals, a.idx_out, 0u,
               0u, 0u, 0u, (const uint32_t*)nullptr, a.mom);
  else
    LW_LAUNCH((k_write<KM_THRESH, OUT_PAIRS, false>), a.n_tasks, st, a.g, a.ef, a.seg_off,
              a.seg_n, a.large_segs, a.tasks, a.st_large, a.pre, a.cap_off, a.pairs, a.vals,
              a.idx_out, 0u,  0u, 0u, 0u, (const uint32_t*)nullptr, a.mom);
}

void unpack_pairs(const int2* gathered, int64_t cap_total, int ws, float* g, const int64_t* seg_off,
                  const int32_t* seg_n, const int64_t* cap_off, const int2* utasks, int n_utasks,
                  hipStream_t st) {
  if (n_utasks == 0) return;
  LW_LAUNCH(k_unpack_pairs, n_utasks, st, gathered, cap_total, ws, g, seg_off, seg_n, cap_off,
            utasks);
}

void unpack_pairs_sgd(const int2* gathered, int64_t cap_total, int ws, const int64_t* seg_off,
                      const int64_t* cap_off, const int4* ftasks, int n_ftasks, const SgdArgs& a,
                      hipStream_t st) {
  if (n_ftasks == 0) return;
  const bool mom = a.momentum != 0.f;
#define LW_USGD(M, N, F) \
  LW_LAUNCH((k_unpack_sgd<M, N, F>), n_ftasks, st, gathered, cap_total, ws, seg_off, cap_off, \
            ftasks, a)
  if (!mom) LW_USGD(false, false, false);
  else if (a.nesterov) { if (a.first_step) LW_USGD(true, true, true); else LW_USGD(true, true, false); }
  else { if (a.first_step) LW_USGD(true, false, true); else LW_USGD(true, false, false); }
#undef LW_USGD
}

void unpack_validx(const float* vals, const int32_t* idx, const int32_t* slot_seg, int64_t nslots,
                   int ws, float* g, const int64_t* seg_off, hipStream_t st) {
  if (nslots == 0) return;
  LW_LAUNCH(k_unpack_validx, (nslots + NT - 1) / NT, st, vals, idx, slot_seg, nslots, ws, g,
            seg_off);
}

void seg_reduce(const QuantArgs& a, bool ef_add, int what, float* out, float2* partial,
                hipStream_t st, bool staged) {
  if (!staged) {      // (staged: quant_stage already wrote every task's partial)
    if (ef_add) LW_LAUNCH((k_partial<true>), a.n_tasks, st, a.g, a.ef, a.seg_off, a.seg_n, a.segs, a.tasks, partial);
    else LW_LAUNCH((k_partial<false>), a.n_tasks, st, a.g, a.ef, a.seg_off, a.seg_n, a.segs, a.tasks, partial);
  }
  LW_LAUNCH(k_finalize, a.nseg, st, partial, a.task_lo, out, what);
}

// Entire-model staging of the quantisers: the per-task (abs-max, sum of squares) partials with the
// error-feedback fold, for tasks [t_lo, t_hi), each into its own slot — the finalize then folds
// the slots in task order, exactly as after one launch.
void quant_stage(const QuantArgs& a, bool ef_add, int t_lo, int t_hi, float2* partial,
                 hipStream_t st) {
  if (t_hi <= t_lo) return;
  if (ef_add) LW_LAUNCH((k_partial<true>), t_hi - t_lo, st, a.g, a.ef, a.seg_off, a.seg_n, a.segs, a.tasks + t_lo, partial + t_lo);
  else LW_LAUNCH((k_partial<false>), t_hi - t_lo, st, a.g, a.ef, a.seg_off, a.seg_n, a.segs, a.tasks + t_lo, partial + t_lo);
}

template <int Q>
static void quant_t(const QuantArgs& a, bool ef, hipStream_t st) {
  if (ef)
    LW_LAUNCH((k_quant<Q, true>), a.n_tasks, st, a.g, a.ef, a.seg_off, a.seg_n, a.segs, a.tasks,
              a.rec_off, a.scale, a.payload, a.nseg, a.qstates, a.gid_base, a.step, a.tag, a.seed0,
              a.seed1, a.step_ptr);
  else
    LW_LAUNCH((k_quant<Q, false>), a.n_tasks, st, a.g, a.ef, a.seg_off, a.seg_n, a.segs, a.tasks,
              a.rec_off, a.scale, a.payload, a.nseg, a.qstates, a.gid_base, a.step, a.tag, a.seed0,
              a.seed1, a.step_ptr);
}

void quantize(const QuantArgs& a, int q, bool ef, hipStream_t st) {
  switch (q) {
    case Q_TERN: quant_t<Q_TERN>(a, ef, st); break;
    case Q_QS8: quant_t<Q_QS8>(a, ef, st); break;
    case Q_QS9: quant_t<Q_QS9>(a, ef, st); break;
    default: quant_t<Q_QS16>(a, ef, st); break;
  }
}

void dequantize(const QuantArgs& a, int q, const uint32_t* gathered, int64_t words_per_rank, int ws,
                hipStream_t st) {
  switch (q) {
    case Q_TERN:
      LW_LAUNCH(k_dequant<Q_TERN>, a.n_tasks, st, gathered, words_per_rank, ws, a.g, a.seg_off,
                a.seg_n, a.segs, a.tasks, a.rec_off, a.nseg, a.qstates);
      break;
    case Q_QS8:
      LW_LAUNCH(k_dequant<Q_QS8>, a.n_tasks, st, gathered, words_per_rank, ws, a.g, a.seg_off,
                a.seg_n, a.segs, a.tasks, a.rec_off, a.nseg, a.qstates);
      break;
    case Q_QS9:
      LW_LAUNCH(k_dequant<Q_QS9>, a.n_tasks, st, gathered, words_per_rank, ws, a.g, a.seg_off,
                a.seg_n, a.segs, a.tasks, a.rec_off, a.nseg, a.qstates);
      break;
    default:
      LW_LAUNCH(k_dequant<Q_QS16>, a.n_tasks, st, gathered, words_per_rank, ws, a.g, a.seg_off,
                a.seg_n, a.segs, a.tasks, a.rec_off, a.nseg, a.qstates);
      break;
  }
}

// ------------------------------------------------------------------------------------------
// Quantised reduce-scatter wire (codecs.py QuantRSCodec). Every rank quantises its whole bucket
// (k_quant); an all-to-all sends rank q only the records of ITS shard of the bucket's groups
// (groups [g0_q, g0_q + ng_q)), each piece laid out [hdr scale words | ng level words x RL |
// (Q_QS9) ng sign words]; rank q dequantises and averages its shard over the W pieces in rank
// order — the arithmetic of k_dequant, so the mean is the all-gather wire's bit for bit before
// its rounding — and writes it as bf16 into the bucket image, which a bf16 all-gather of the
// shards then completes on every rank. gtab[g] = (segment, bucket element offset, valid
// elements, 0) of global group g.
// ------------------------------------------------------------------------------------------
template <int Q>
__global__ __launch_bounds__(NT) void k_dequant_shard(const uint32_t* __restrict__ recv, int64_t wpr,
                                                      int ws, int hdr, const int4* __restrict__ gtab,
                                                      int64_t g0, int64_t ng, int qstates,
                                                      uint16_t* __restrict__ out, int64_t n_out) {
  // no FMA contraction: each product and sum rounds on its own, as the CPU mirror's numpy does.
  // (The pragma only reaches operators written here: the __f*_rn header helpers carry the file's
  // fast contraction into the inlined code, where they were fused back into FMAs.)
#pragma clang fp contract(off)
  const int64_t j = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (j >= ng) return;
  const int4 gt = gtab[g0 + j];
  // (a malformed table entry writes nothing rather than out of bounds)
  if (gt.x < 0 || gt.x >= hdr || gt.y < 0 || gt.z < 0 || gt.z > EPT || gt.y + gt.z > n_out) return;
  constexpr int RL = Q == Q_TERN ? 2 : (Q == Q_QS16 ? 16 : 8);
  float acc[EPT];
#pragma unroll
  for (int k = 0; k < EPT; ++k) acc[k] = 0.f;
  for (int r = 0; r < ws; ++r) {
    const uint32_t* P = recv + (int64_t)r * wpr;
    const float sc = __uint_as_float(P[gt.x]);
    const uint32_t* rec = P + hdr + j * RL;
    if (Q == Q_TERN) {
      const uint2 w = *reinterpret_cast<const uint2*>(rec);
#pragma unroll
      for (int k = 0; k < EPT; ++k) {
        const uint32_t c = ((k < 16 ? w.x : w.y) >> (2 * (k & 15))) & 3u;
        acc[k] = acc[k] + (c == 1u ? sc : (c == 2u ? -sc : 0.f));
      }
    } else if (Q == Q_QS8) {
      const uint4* o = reinterpret_cast<const uint4*>(rec);
      const uint4 a = o[0], b = o[1];
      const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
      for (int k = 0; k < EPT; ++k) {
        const int l = (int)(int8_t)((w[k >> 2] >> (8 * (k & 3))) & 0xff);
        const float sg = l > 0 ? 1.f : (l < 0 ? -1.f : 0.f);
        acc[k] = acc[k] + sg * sc * ((float)(l < 0 ? -l : l) / (float)qstates);
      }
    } else if (Q == Q_QS9) {
      const uint4* o = reinterpret_cast<const uint4*>(rec);
      const uint4 a = o[0], b = o[1];
      const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      const uint32_t sgn = P[hdr + ng * 8 + j];
#pragma unroll
      for (int k = 0; k < EPT; ++k) {
        const int l = (int)((w[k >> 2] >> (8 * (k & 3))) & 0xff);
        const float sg = l == 0 ? 0.f : (((sgn >> k) & 1u) ? -1.f : 1.f);
        acc[k] = acc[k] + sg * sc * ((float)l / (float)qstates);
      }
    } else {
      const uint4* o = reinterpret_cast<const uint4*>(rec);
      uint32_t w[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 x = o[q];
        w[4 * q] = x.x; w[4 * q + 1] = x.y; w[4 * q + 2] = x.z; w[4 * q + 3] = x.w;
      }
#pragma unroll
      for (int k = 0; k < EPT; ++k) {
        const int l = (int)(int16_t)((w[k >> 1] >> (16 * (k & 1))) & 0xffff);
        const float sg = l > 0 ? 1.f : (l < 0 ? -1.f : 0.f);
        acc[k] = acc[k] + sg * sc * ((float)(l < 0 ? -l : l) / (float)qstates);
      }
    }
  }
  const float fws = (float)ws;
  // (uncontracted adds / products, correctly rounded quotients, so the CPU mirror —
  // codecs.py QuantRSCodec.reduce_shard — reproduces every shard bit for bit)
  uint16_t* op = out + gt.y;
  if (gt.z == EPT && (gt.y & 7) == 0) {
#pragma unroll
    for (int q = 0; q < EPT / 8; ++q) {
      uint32_t w[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        w[k] = (uint32_t)ElemBF16::rne(acc[8 * q + 2 * k] / fws) |
               ((uint32_t)ElemBF16::rne(acc[8 * q + 2 * k + 1] / fws) << 16);
      reinterpret_cast<uint4*>(op)[q] = make_uint4(w[0], w[1], w[2], w[3]);
    }
  } else {
    for (int k = 0; k < gt.z; ++k) op[k] = ElemBF16::rne(acc[k] / fws);
  }
}

__global__ __launch_bounds__(NT) void k_bf16_expand(const uint16_t* __restrict__ in,
                                                    float* __restrict__ out, int64_t n) {
  const int64_t step = (int64_t)gridDim.x * NT * 8;
  for (int64_t i = ((int64_t)blockIdx.x * NT + threadIdx.x) * 8; i < n; i += step) {
    if (i + 8 <= n) {
      const uint4 v = *reinterpret_cast<const uint4*>(in + i);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      float4* o = reinterpret_cast<float4*>(out + i);
      o[0] = make_float4(ElemBF16::lo(w[0]), ElemBF16::hi(w[0]), ElemBF16::lo(w[1]), ElemBF16::hi(w[1]));
      o[1] = make_float4(ElemBF16::lo(w[2]), ElemBF16::hi(w[2]), ElemBF16::lo(w[3]), ElemBF16::hi(w[3]));
    } else {
      for (int64_t k = i; k < n; ++k) out[k] = ElemBF16::f(in[k]);
    }
  }
}

void dequantize_shard(int q, const uint32_t* recv, int64_t wpr, int ws, int hdr, const int4* gtab,
                      int64_t g0, int64_t ng, int qstates, uint16_t* out, int64_t n_out,
                      hipStream_t st) {
  if (ng <= 0) return;
  const int64_t grid = (ng + NT - 1) / NT;
  switch (q) {
    case Q_TERN: LW_LAUNCH(k_dequant_shard<Q_TERN>, grid, st, recv, wpr, ws, hdr, gtab, g0, ng, qstates, out, n_out); break;
    case Q_QS8: LW_LAUNCH(k_dequant_shard<Q_QS8>, grid, st, recv, wpr, ws, hdr, gtab, g0, ng, qstates, out, n_out); break;
    case Q_QS9: LW_LAUNCH(k_dequant_shard<Q_QS9>, grid, st, recv, wpr, ws, hdr, gtab, g0, ng, qstates, out, n_out); break;
    default: LW_LAUNCH(k_dequant_shard<Q_QS16>, grid, st, recv, wpr, ws, hdr, gtab, g0, ng, qstates, out, n_out); break;
  }
}

void bf16_expand(const uint16_t* in, float* out, int64_t n, hipStream_t st) {
  if (n <= 0) return;
  int64_t grid = (n + NT * 8 - 1) / (NT * 8);
  grid = grid > 2048 ? 2048 : grid;
  LW_LAUNCH(k_bf16_expand, grid, st, in, out, n);
}

// Simulated wire time (parallel/loopback.py wire model, train/simworld.py): `nwg` single-wave
// workgroups each hold a CU slot — as RCCL's channel workgroups do during a real transfer — until
// `ticks` of the constant wall clock have passed since it started, sleeping between reads. Every
// wave leaves once its own deadline passes, so the grid always drains.
__global__ __launch_bounds__(64) void k_wire_wait(uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

void wire_wait(double us, int nwg, hipStream_t st) {
  static int khz = 0;
  if (khz == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
      khz = 100000;                              // the 100 MHz constant clock of CDNA3/4
  }
  if (us <= 0.0 || nwg <= 0) return;
  const uint64_t ticks = (uint64_t)(us * (double)khz / 1000.0);
  hipLaunchKernelGGL(k_wire_wait, dim3(nwg), dim3(64), 0, st, ticks);
}

}  // namespace lw
