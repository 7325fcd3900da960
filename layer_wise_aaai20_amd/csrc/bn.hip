// Fused BatchNorm (+ residual add) (+ ReLU) for NHWC (channels_last) activations on gfx950.
//
// The reference's ResNets run cuDNN BatchNorm, then a separate ReLU, then a separate residual add
// (IMAGENET/training/resnet.py:60-80, CIFAR10/dawn.py:23-35): on MI355X those glue ops were 62 % of
// a ResNet-50 step (profiles/r1_baseline_summary.txt). Here a BN layer costs two passes forward
// (per-channel sum/sumsq, then normalise+affine+add+ReLU) and two backward (per-channel reductions
// of dy' and dy'·x̂ with the ReLU mask folded in, then dx and the residual gradient) — SURVEY.md N16.
//
// Data layout: x is [M = N*H*W, C] with C contiguous, C % 8 == 0. Each lane moves 8 channels (one
// 16-byte bf16 load). Reductions go to per-block partial sums in a fixed order (deterministic), and
// a finalize kernel folds them in fp64.
#include "common.h"
#include "lw_kernels.h"
#include "elem16.h"
#include <cstdlib>

namespace lw {

constexpr int BNT = 256;

template <typename T> struct V8;
template <> struct V8<uint16_t> {
  // raw 16-byte form, so a loop can have the next rows' loads in flight while it converts and
  // accumulates the current ones
  typedef uint4 Raw;
  static __device__ __forceinline__ Raw ld(const uint16_t* p) { return *reinterpret_cast<const uint4*>(p); }
  static __device__ __forceinline__ Raw zero() { return make_uint4(0u, 0u, 0u, 0u); }
  static __device__ __forceinline__ void cvt(const Raw& v, float f[8]) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f[2 * k] = hlo(w[k]);
      f[2 * k + 1] = hhi(w[k]);
    }
  }
  static __device__ __forceinline__ void load(const uint16_t* p, float f[8]) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f[2 * k] = hlo(w[k]);
      f[2 * k + 1] = hhi(w[k]);
    }
  }
  static __device__ __forceinline__ void store(uint16_t* p, const float f[8]) {
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      w[k] = (uint32_t)f2h(f[2 * k]) | ((uint32_t)f2h(f[2 * k + 1]) << 16);
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
};
template <> struct V8<float> {
  struct Raw { float4 a, b; };
  static __device__ __forceinline__ Raw ld(const float* p) {
    return Raw{reinterpret_cast<const float4*>(p)[0], reinterpret_cast<const float4*>(p)[1]};
  }
  static __device__ __forceinline__ Raw zero() {
    return Raw{make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
  }
  static __device__ __forceinline__ void cvt(const Raw& v, float f[8]) {
    f[0] = v.a.x; f[1] = v.a.y; f[2] = v.a.z; f[3] = v.a.w;
    f[4] = v.b.x; f[5] = v.b.y; f[6] = v.b.z; f[7] = v.b.w;
  }
  static __device__ __forceinline__ void load(const float* p, float f[8]) {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* p, const float f[8]) {
    reinterpret_cast<float4*>(p)[0] = make_float4(f[0], f[1], f[2], f[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(f[4], f[5], f[6], f[7]);
  }
};

// ------------------------------------------------------------------------------------------
// Column reductions over [M, C]. MODE 0 (forward): (Σx, Σx²). MODE 1 (backward):
// (Σdy', Σdy'·(x-mean)) with dy' = relu ? dy·[y>0] : dy.
// Thread (g, r): channel group g (8 channels), row lane r of R = BNT/G. 4 rows in flight per lane.
// partial: [gridDim.x][2C]
// ------------------------------------------------------------------------------------------
// RELU: 0 none, 1 mask from the saved output y, 2 mask recomputed from x: x*scale+shift > 0
// (bit-identical to the forward's test, which evaluated the same fp32 expression), 3 mask from
// the 1-bit-per-element ReLU bitmap the forward apply wrote (1/16 of the bytes of y).
__device__ __forceinline__ void mask_bits(float d[8], uint32_t bits) {
#pragma unroll
  for (int k = 0; k < 8; ++k) d[k] = ((bits >> k) & 1u) ? d[k] : 0.f;
}

// DUAL (MODE 1): a second BN whose input x2 received the same gradient dy and ReLU mask (the
// downsample shortcut's BN next to BN3 in a bottleneck): Σdy' is shared, Σdy'·(x2−mean2) goes to
// partial2 ([2][C][nb] like partial) — one pass over dy and the bitmap for both BNs.
template <typename T, int MODE, int RELU, int U, bool DUAL = false>
__global__ __launch_bounds__(BNT) void k_bn_reduce(const T* __restrict__ x, const T* __restrict__ dy,
                                                   const T* __restrict__ y,
                                                   const uint8_t* __restrict__ bits,
                                                   const float* __restrict__ mean,
                                                   const float* __restrict__ fscale,
                                                   const float* __restrict__ fshift, int64_t M,
                                                   int C, int64_t rows_per_block,
                                                   float* __restrict__ partial,
                                                   const T* __restrict__ x2 = nullptr,
                                                   const float* __restrict__ mean2 = nullptr,
                                                   float* __restrict__ partial2 = nullptr) {
  static_assert(!DUAL || MODE == 1, "dual reduce: backward only");
  __shared__ float sa[BNT * 8];
  __shared__ float sb[BNT * 8];
  __shared__ float sb2[DUAL ? BNT * 8 : 1];
  // blockIdx.y selects a slice of Cb channels (reduce_geometry): a block reads Cb-wide row
  // segments, so it writes 2*Cb partial sums instead of 2*C scattered ones (at C = 2048 the
  // whole-row form spent most of its time on 4096 strided partial stores per block)
  const int Cb = C / (int)gridDim.y, c_off = (int)blockIdx.y * Cb;
  const int G = Cb / 8, GC = C / 8;
  const int R = BNT / G;                    // rows processed per iteration (>= 1)
  const int g = threadIdx.x % G, r = threadIdx.x / G;
  const int gc = c_off / 8 + g;             // this thread's channel group within the full row
  const bool active = r < R;
  float a[8], b[8], mu[8], fs[8], fh[8], b2[8], mu2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a[k] = 0.f; b[k] = 0.f; mu[k] = 0.f; fs[k] = 0.f; fh[k] = 0.f; b2[k] = 0.f; mu2[k] = 0.f;
  }
  if (MODE == 1 && active) {
#pragma unroll
    for (int k = 0; k < 8; ++k) mu[k] = mean[gc * 8 + k];
    if (DUAL) {
#pragma unroll
      for (int k = 0; k < 8; ++k) mu2[k] = mean2[gc * 8 + k];
    }
    if (RELU == 2) {
#pragma unroll
      for (int k = 0; k < 8; ++k) { fs[k] = fscale[gc * 8 + k]; fh[k] = fshift[gc * 8 + k]; }
    }
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(r0 + rows_per_block, M);
  if (active) {
    using V = V8<T>;
    typedef typename V::Raw Raw;
    const T* xp = x + gc * 8;
    const T* dp = dy + gc * 8;
    const T* yp = y + gc * 8;
    const T* x2p = DUAL ? x2 + gc * 8 : nullptr;
    // Software-pipelined: the U rows of the next iteration are loaded (raw, predicated: rows past
    // r1 read as zero and add nothing) before the current U rows are converted and accumulated.
    // (with DUAL, the y slots carry x2: a dual reduce always takes its mask from the bitmap)
    static_assert(!DUAL || RELU == 3, "dual reduce: bitmap mask");
    Raw cx[U], cd[U], cy[U];
    uint32_t cb[U];
    auto fetch = [&](int64_t row0, Raw (&fx)[U], Raw (&fd)[U], Raw (&fy)[U], uint32_t (&fb)[U]) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t rw = row0 + u * R;
        const bool in = rw < r1;
        fx[u] = in ? V::ld(xp + rw * C) : V::zero();
        if (MODE == 1) {
          fd[u] = in ? V::ld(dp + rw * C) : V::zero();
          if (RELU == 1) fy[u] = in ? V::ld(yp + rw * C) : V::zero();
          if (DUAL) fy[u] = in ? V::ld(x2p + rw * C) : V::zero();
          if (RELU == 3) fb[u] = in ? (uint32_t)bits[rw * GC + gc] : 0u;
        }
      }
    };
    int64_t row = r0 + r;
    fetch(row, cx, cd, cy, cb);
    for (; row < r1; row += U * R) {
      Raw nx[U], nd[U], ny[U];
      uint32_t nb8[U];
      const bool more = row + U * R < r1;
      if (more) fetch(row + U * R, nx, nd, ny, nb8);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float xv[8];
        V::cvt(cx[u], xv);
        if (MODE == 0) {
#pragma unroll
          for (int k = 0; k < 8; ++k) { a[k] += xv[k]; b[k] += xv[k] * xv[k]; }
        } else {
          float d[8];
          V::cvt(cd[u], d);
          if (RELU == 1) {
            float yv[8];
            V::cvt(cy[u], yv);
#pragma unroll
            for (int k = 0; k < 8; ++k) d[k] = yv[k] > 0.f ? d[k] : 0.f;
          } else if (RELU == 2) {
#pragma unroll
            for (int k = 0; k < 8; ++k) d[k] = fmaf(xv[k], fs[k], fh[k]) > 0.f ? d[k] : 0.f;
          } else if (RELU == 3) {
            mask_bits(d, cb[u]);
          }
#pragma unroll
          for (int k = 0; k < 8; ++k) { a[k] += d[k]; b[k] += d[k] * (xv[k] - mu[k]); }
          if (DUAL) {
            float x2v[8];
            V::cvt(cy[u], x2v);
#pragma unroll
            for (int k = 0; k < 8; ++k) b2[k] += d[k] * (x2v[k] - mu2[k]);
          }
        }
      }
      if (more) {
#pragma unroll
        for (int u = 0; u < U; ++u) { cx[u] = nx[u]; cd[u] = nd[u]; cy[u] = ny[u]; cb[u] = nb8[u]; }
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sa[r * Cb + g * 8 + k] = a[k];
      sb[r * Cb + g * 8 + k] = b[k];
      if (DUAL) sb2[r * Cb + g * 8 + k] = b2[k];
    }
  }
  __syncthreads();
  const int64_t nb = gridDim.x;
  for (int c = threadIdx.x; c < Cb; c += BNT) {
    float s1 = 0.f, s2 = 0.f, s3 = 0.f;
    for (int q = 0; q < R; ++q) {
      s1 += sa[q * Cb + c];
      s2 += sb[q * Cb + c];
      if (DUAL) s3 += sb2[q * Cb + c];
    }
    partial[(int64_t)(c_off + c) * nb + blockIdx.x] = s1;       // channel-major: [2][C][nb]
    partial[((int64_t)C + c_off + c) * nb + blockIdx.x] = s2;
    if (DUAL) {
      partial2[(int64_t)(c_off + c) * nb + blockIdx.x] = s1;
      partial2[((int64_t)C + c_off + c) * nb + blockIdx.x] = s3;
    }
  }
}

// Fold the block partials: one wave per channel, lanes stride over blocks (coalesced, fixed
// order), then a fixed butterfly in fp64. Lane 0 of each wave gets the sums.
// rstride > 0: `partial` is instead the GEMM epilogue's statistics rows themselves, [nblocks][rstride]
// (column c: Σv, C + c: Σv²) — k_colsum with one row per block wrote exactly those values, so
// the fold is the same bit for bit without that launch.
__device__ __forceinline__ bool fold_channel(const float* __restrict__ partial, int nblocks, int C,
                                             int c, double& s1, double& s2, int rstride = 0);
__device__ __forceinline__ bool fold_partials(const float* __restrict__ partial, int nblocks, int C,
                                              double& s1, double& s2, int& c, int rstride = 0) {
  c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C) return false;
  return fold_channel(partial, nblocks, C, c, s1, s2, rstride);
}
__device__ __forceinline__ bool fold_channel(const float* __restrict__ partial, int nblocks, int C,
                                             int c, double& s1, double& s2, int rstride) {
  const int lane = threadIdx.x & 63;
  const int64_t bs = rstride > 0 ? rstride : 1;          // element stride between blocks
  const float* p1 = partial + (rstride > 0 ? (int64_t)c : (int64_t)c * nblocks);
  const float* p2 = partial + (rstride > 0 ? (int64_t)C + c : ((int64_t)C + c) * nblocks);
  float a = 0.f, b = 0.f;
  // 16 strided loads per lane issued together, then added in block order (a plain strided loop
  // waited for each load in turn: ~8 µs of HBM latency per launch)
  for (int base = 0; base < nblocks; base += 16 * 64) {
    float va[16], vb[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int blk = base + u * 64 + lane;
      va[u] = blk < nblocks ? p1[blk * bs] : 0.f;
      vb[u] = blk < nblocks ? p2[blk * bs] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) { a += va[u]; b += vb[u]; }
  }
  double da = a, db = b;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    da += __shfl_xor(da, o, 64);
    db += __shfl_xor(db, o, 64);
  }
  s1 = da;
  s2 = db;
  return lane == 0;
}

// mean / invstd / scale / shift (+ running statistics) of channel c from its folded sums
__device__ __forceinline__ void finalize_fwd_channel(int c, double s, double q, int64_t M,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float eps,
                                                     float momentum, float* __restrict__ rmean,
                                                     float* __restrict__ rvar,
                                                     float* __restrict__ mean_out,
                                                     float* __restrict__ invstd_out,
                                                     float* __restrict__ scale,
                                                     float* __restrict__ shift) {
  const double mean = s / (double)M;
  double var = q / (double)M - mean * mean;
  var = var < 0.0 ? 0.0 : var;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  mean_out[c] = (float)mean;
  invstd_out[c] = invstd;
  scale[c] = gm * invstd;
  shift[c] = bt - (float)mean * gm * invstd;
  if (rmean) {
    const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
    rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
    rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * unbiased);
  }
}

__global__ __launch_bounds__(256) void k_bn_finalize_fwd(
    const float* __restrict__ partial, int nblocks, int C, int64_t M,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float momentum,
    float* __restrict__ rmean, float* __restrict__ rvar, float* __restrict__ mean_out,
    float* __restrict__ invstd_out, float* __restrict__ scale, float* __restrict__ shift,
    int rstride) {
  double s, q;
  int c;
  if (!fold_partials(partial, nblocks, C, s, q, c, rstride)) return;
  const double mean = s / (double)M;
  double var = q / (double)M - mean * mean;
  var = var < 0.0 ? 0.0 : var;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  mean_out[c] = (float)mean;
  invstd_out[c] = invstd;
  scale[c] = gm * invstd;
  shift[c] = bt - (float)mean * gm * invstd;
  if (rmean) {
    const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
    rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
    rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * unbiased);
  }
}

// Rows [R][W] fp32 → per-block column sums, channel-major partial [W][gridDim.x] (the layout
// k_bn_finalize_fwd folds). Folds the per-M-tile statistics rows a GEMM epilogue wrote
// (gemm.hip EPI_STATS, W = 2C: Σv then Σv²); rows are summed in order (deterministic).
__global__ __launch_bounds__(256) void k_colsum(const float* __restrict__ rows, int64_t R, int W,
                                                int64_t rows_per_block,
                                                float* __restrict__ partial) {
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(r0 + rows_per_block, R);
  for (int c = threadIdx.x; c < W; c += 256) {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int64_t r = r0;
    for (; r + 3 < r1; r += 4) {
      s0 += rows[r * W + c];
      s1 += rows[(r + 1) * W + c];
      s2 += rows[(r + 2) * W + c];
      s3 += rows[(r + 3) * W + c];
    }
    for (; r < r1; ++r) s0 += rows[r * W + c];
    partial[(int64_t)c * gridDim.x + blockIdx.x] = (s0 + s1) + (s2 + s3);
  }
}

// Thread-constant channel group: the grid-stride step is a multiple of G = C/8 (apply_grid), so
// a thread always touches the same 8 channels and keeps their coefficients in registers.
// ReLU bitmap of 8 outputs: bit k set iff the STORED (bf16-rounded) value is > 0, i.e. exactly
// the test the backward would apply to the saved output.
__device__ __forceinline__ uint8_t relu_bits(const float v[8]) {
  uint32_t b = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) b |= (h2f(f2h(v[k])) > 0.f ? 1u : 0u) << k;
  return (uint8_t)b;
}

// RES: 0 none, 1 plain residual add, 2 residual through its own BatchNorm affine (the downsample
// branch of a ResNet block: y = relu(x*scale+shift + r*rscale+rshift), the normalised shortcut is
// never materialised).
template <typename T, int RES, bool RELU>
__global__ __launch_bounds__(BNT) void k_bn_apply(const T* __restrict__ x, const T* __restrict__ res,
                                                  T* __restrict__ y,
                                                  const float* __restrict__ scale,
                                                  const float* __restrict__ shift,
                                                  const float* __restrict__ rscale,
                                                  const float* __restrict__ rshift,
                                                  uint8_t* __restrict__ bits_out, int64_t n8,
                                                  int C) {
  const int G = C / 8;
  const int64_t t0 = (int64_t)blockIdx.x * BNT + threadIdx.x;
  const int64_t step = (int64_t)gridDim.x * BNT;
  const int c0 = (int)(t0 % G) * 8;
  float sc[8], sh[8], rs[8], rh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc[k] = scale[c0 + k]; sh[k] = shift[c0 + k];
    rs[k] = RES == 2 ? rscale[c0 + k] : 1.f;
    rh[k] = RES == 2 ? rshift[c0 + k] : 0.f;
  }
  int64_t i = t0;
  for (; i + step < n8; i += 2 * step) {
    float v[2][8], rr[2][8];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      V8<T>::load(x + (i + u * step) * 8, v[u]);
      if (RES) V8<T>::load(res + (i + u * step) * 8, rr[u]);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float t = fmaf(v[u][k], sc[k], sh[k]);
        if (RES == 1) t += rr[u][k];
        if (RES == 2) t += fmaf(rr[u][k], rs[k], rh[k]);
        if (RELU) t = fmaxf(t, 0.f);
        v[u][k] = t;
      }
      V8<T>::store(y + (i + u * step) * 8, v[u]);
      if (RELU && bits_out) bits_out[i + u * step] = relu_bits(v[u]);
    }
  }
  if (i < n8) {
    float v[8], rr[8];
    V8<T>::load(x + i * 8, v);
    if (RES) V8<T>::load(res + i * 8, rr);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float t = fmaf(v[k], sc[k], sh[k]);
      if (RES == 1) t += rr[k];
      if (RES == 2) t += fmaf(rr[k], rs[k], rh[k]);
      if (RELU) t = fmaxf(t, 0.f);
      v[k] = t;
    }
    V8<T>::store(y + i * 8, v);
    if (RELU && bits_out) bits_out[i] = relu_bits(v);
  }
}

__global__ __launch_bounds__(256) void k_bn_finalize_bwd(
    const float* __restrict__ partial, int nblocks, int C, int64_t M,
    const float* __restrict__ gamma, const float* __restrict__ mean,
    const float* __restrict__ invstd, float* __restrict__ dgamma, float* __restrict__ dbeta,
    float* __restrict__ A, float* __restrict__ B, float* __restrict__ Cc, int training,
    int accum, int rstride) {
  double s1, s2;
  int c;
  if (!fold_partials(partial, nblocks, C, s1, s2, c, rstride)) return;
  const double is = invstd[c];
  const double gm = gamma ? gamma[c] : 1.0;
  if (dbeta) dbeta[c] = accum ? dbeta[c] + (float)s1 : (float)s1;
  if (dgamma) dgamma[c] = accum ? dgamma[c] + (float)(s2 * is) : (float)(s2 * is);
  const double a = gm * is;
  if (!training) {             // running statistics are constants: dx = gamma*invstd*dy'
    A[c] = (float)a;
    B[c] = 0.f;
    Cc[c] = 0.f;
    return;
  }
  const double bb = -gm * is * is * is * s2 / (double)M;
  A[c] = (float)a;
  B[c] = (float)bb;
  Cc[c] = (float)(-a * s1 / (double)M - bb * (double)mean[c]);
}

// dx = A*dy' + B*x + C ; dres = dy'
template <typename T, int RELU, bool DRES>
__global__ __launch_bounds__(BNT) void k_bn_bwd_apply(const T* __restrict__ x, const T* __restrict__ dy,
                                                      const T* __restrict__ y,
                                                      const uint8_t* __restrict__ bits,
                                                      const float* __restrict__ fscale,
                                                      const float* __restrict__ fshift,
                                                      const float* __restrict__ A,
                                                      const float* __restrict__ B,
                                                      const float* __restrict__ Cc,
                                                      T* __restrict__ dx, T* __restrict__ dres,
                                                      int64_t n8, int C) {
  const int G = C / 8;
  const int64_t t0 = (int64_t)blockIdx.x * BNT + threadIdx.x;
  const int64_t step = (int64_t)gridDim.x * BNT;
  const int c0 = (int)(t0 % G) * 8;
  float ca[8], cb[8], cc[8], fs[8], fh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    ca[k] = A[c0 + k]; cb[k] = B[c0 + k]; cc[k] = Cc[c0 + k];
    fs[k] = RELU == 2 ? fscale[c0 + k] : 0.f;
    fh[k] = RELU == 2 ? fshift[c0 + k] : 0.f;
  }
  for (int64_t i0 = t0; i0 < n8; i0 += step) {
    const int64_t i = i0;
    const int64_t off = i * 8;
    float xv[8], d[8];
    V8<T>::load(x + off, xv);
    V8<T>::load(dy + off, d);
    if (RELU == 1) {
      float yv[8];
      V8<T>::load(y + off, yv);
#pragma unroll
      for (int k = 0; k < 8; ++k) d[k] = yv[k] > 0.f ? d[k] : 0.f;
    } else if (RELU == 2) {
#pragma unroll
      for (int k = 0; k < 8; ++k) d[k] = fmaf(xv[k], fs[k], fh[k]) > 0.f ? d[k] : 0.f;
    } else if (RELU == 3) {
      mask_bits(d, bits[i]);
    }
    if (DRES) V8<T>::store(dres + off, d);
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = ca[k] * d[k] + cb[k] * xv[k] + cc[k];
    V8<T>::store(dx + off, o);
  }
}

// The two BN backwards of k_bn_reduce DUAL in one pass: dx = A*dy' + B*x + C and
// dx2 = A2*dy' + B2*x2 + C2 with dy' = dy·bit (dy and the bitmap read once).
__global__ __launch_bounds__(BNT) void k_bn_bwd_apply_dual(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ x2,
    const uint16_t* __restrict__ dy, const uint8_t* __restrict__ bits,
    const float* __restrict__ A, const float* __restrict__ B, const float* __restrict__ Cc,
    const float* __restrict__ A2, const float* __restrict__ B2, const float* __restrict__ Cc2,
    uint16_t* __restrict__ dx, uint16_t* __restrict__ dx2, int64_t n8, int C) {
  const int G = C / 8;
  const int64_t t0 = (int64_t)blockIdx.x * BNT + threadIdx.x;
  const int64_t step = (int64_t)gridDim.x * BNT;
  const int c0 = (int)(t0 % G) * 8;
  float ca[8], cb[8], cc[8], ca2[8], cb2[8], cc2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    ca[k] = A[c0 + k]; cb[k] = B[c0 + k]; cc[k] = Cc[c0 + k];
    ca2[k] = A2[c0 + k]; cb2[k] = B2[c0 + k]; cc2[k] = Cc2[c0 + k];
  }
  for (int64_t i0 = t0; i0 < n8; i0 += step) {
    const int64_t i = i0;
    const int64_t off = i * 8;
    float xv[8], x2v[8], d[8];
    V8<uint16_t>::load(x + off, xv);
    V8<uint16_t>::load(x2 + off, x2v);
    V8<uint16_t>::load(dy + off, d);
    mask_bits(d, bits[i]);
    float o[8], o2[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      o[k] = ca[k] * d[k] + cb[k] * xv[k] + cc[k];
      o2[k] = ca2[k] * d[k] + cb2[k] * x2v[k] + cc2[k];
    }
    V8<uint16_t>::store(dx + off, o);
    V8<uint16_t>::store(dx2 + off, o2);
  }
}

// ------------------------------------------------------------------------------------------
// Geometry (measured constants; round 6 removed the environment knobs that tuned them).
// Reduce grid: (row blocks) x (channel slices of Cb = 128 channels when C is a multiple of 128,
// else the whole row), about kReduceBlocks workgroups in total; nblocks (row blocks) is the number
// of partial sums per channel the finalize folds. 4 rows in flight per lane (8 measured slower:
// profiles/r6/bn_stream_probe_a.txt, 143 vs 167 us at the layer-1 shape).
constexpr int64_t kReduceBlocks = 512;
constexpr int kReduceUnroll = 4;
static int reduce_slices(int C) { return (C > 128 && C % 128 == 0) ? C / 128 : 1; }

// The dual reduce (three activation streams + the bitmap) on tensors beyond the Infinity Cache:
// half the workgroups, 228 vs 247 us at the layer-1 shape (profiles/r6/bn_stream_probe2.txt)
constexpr int64_t kDualReduceBlocks = 256;
constexpr int64_t kDualFewBlocksMin = int64_t(128) << 20;   // elements per stream

static void reduce_geometry(int64_t M, int C, int64_t& rows_per_block, int& nblocks,
                            int64_t target = kReduceBlocks) {
  const int nsl = reduce_slices(C);
  const int G = C / nsl / 8;
  const int R = BNT / G;
  const int64_t rb = (target + nsl - 1) / nsl;
  int64_t rpb = (M + rb - 1) / rb;
  rpb = (rpb + R - 1) / R * R;
  rpb = rpb < R ? R : rpb;
  rows_per_block = rpb;
  nblocks = (int)((M + rpb - 1) / rpb);
}

// GEMM statistics rows folded by the finalize itself up to this many rows (k_colsum with one row
// per block wrote exactly those values), else summed by k_colsum into at most kColsumBlocks
// partials first
constexpr int64_t kColsumDirectMax = 1024;
constexpr int kColsumBlocks = 1024;
int colsum_blocks(int64_t rows) { return (int)(rows < kColsumBlocks ? rows : kColsumBlocks); }

int bn_reduce_blocks(int64_t M, int C) {
  int64_t rpb;
  int nb;
  reduce_geometry(M, C, rpb, nb);
  return nb;
}

// grid with (gridDim * BNT) % G == 0 so every thread keeps one channel group. `cap` workgroups at
// most: fewer, longer grid-stride sweeps keep each CU's accesses within fewer DRAM pages. Measured
// on the 411 MB layer-1 tensors (scripts/probes/bn_stream_probe.hip, profiles/r6/bn_stream_probe*):
// the residual forward apply 279 -> 221 us at 512 workgroups instead of 4096, the backward apply
// 238 -> 224 us at 1024 (512 starves it of loads in flight: 287 us).
constexpr int kApplyFwdGrid = 512, kApplyBwdGrid = 1024;
static int apply_grid(int64_t n8, int C, int cap) {
  const int G = C / 8;
  int q = G;                                   // blocks must be a multiple of G / gcd(G, BNT)
  int a = G, b = BNT;
  while (b) { const int t = a % b; a = b; b = t; }
  q = G / a;
  int64_t g = (n8 + BNT - 1) / BNT;
  g = g > cap ? cap : (g < 1 ? 1 : g);
  g = (g + q - 1) / q * q;
  return (int)g;
}

template <typename T>
static void bn_apply_t(const BNArgs& a, hipStream_t st) {
  const T* x = static_cast<const T*>(a.x);
  const T* res = static_cast<const T*>(a.res);
  T* y = static_cast<T*>(a.y);
  const int64_t n8 = a.M * a.C / 8;
  const dim3 grid(apply_grid(n8, a.C, kApplyFwdGrid)), block(BNT);
#define LW_AP(R, L)                                                                              \
  hipLaunchKernelGGL((k_bn_apply<T, R, L>), grid, block, 0, st, x, res, y, a.scale, a.shift,     \
                     a.res_scale, a.res_shift, a.bits, n8, a.C)
  const int rm = !res ? 0 : (a.res_scale ? 2 : 1);
  if (rm == 2) { if (a.relu) LW_AP(2, true); else LW_AP(2, false); }
  else if (rm == 1) { if (a.relu) LW_AP(1, true); else LW_AP(1, false); }
  else { if (a.relu) LW_AP(0, true); else LW_AP(0, false); }
#undef LW_AP
}

// Batch statistics -> mean / invstd / scale / shift (+ running-stat update). With
// a.stats_blocks > 0 the per-block partial sums are already in a.partial (written by the epilogue
// of the producing GEMM, gemm.hip EPI_STATS) and only the finalize runs.
template <typename T>
static void bn_stats_t(const BNArgs& a, hipStream_t st) {
  int nb = a.stats_blocks;
  const float* part = a.partial;
  int rstride = 0;
  if (a.stat_rows) {                      // GEMM epilogue rows [R][2C] -> [2C][nb]
    const int64_t R = a.stats_rows_n;
    nb = colsum_blocks(R);
    const int64_t rpb = (R + nb - 1) / nb;
    nb = (int)((R + rpb - 1) / rpb);
    if (R <= kColsumDirectMax) {
      // few rows: the finalize folds the rows where they are, one launch fewer. Up to 1024 rows
      // k_colsum ran one row per block, so the sums are its own bit for bit (layers 3-4 of a
      // ResNet-50, 29 BatchNorms: 11,332-11,372 -> 11,439-11,465 img/s on one box; a cap of
      // 2048 / 8192 rows measured 11,429-11,438 / 11,375, profiles/r5/colsum_direct_ab.jsonl)
      part = a.stat_rows;
      rstride = 2 * a.C;
      nb = (int)R;
    } else {
      hipLaunchKernelGGL(k_colsum, dim3(nb), dim3(256), 0, st, a.stat_rows, R, 2 * a.C, rpb,
                         a.partial);
    }
  } else if (nb <= 0) {
    int64_t rpb;
    reduce_geometry(a.M, a.C, rpb, nb);
    auto kern = k_bn_reduce<T, 0, 0, kReduceUnroll>;
    hipLaunchKernelGGL(kern, dim3(nb, reduce_slices(a.C)), dim3(BNT), 0, st, static_cast<const T*>(a.x),
                       (const T*)nullptr, (const T*)nullptr, (const uint8_t*)nullptr,
                       (const float*)nullptr,
                       (const float*)nullptr, (const float*)nullptr, a.M, a.C, rpb, a.partial,
                       (const T*)nullptr, (const float*)nullptr, (float*)nullptr);
  }
  hipLaunchKernelGGL(k_bn_finalize_fwd, dim3((a.C + 3) / 4), dim3(256), 0, st, part, nb,
                     a.C, a.M, a.gamma, a.beta, a.eps, a.momentum, a.rmean, a.rvar, a.mean,
                     a.invstd, a.scale, a.shift, rstride);
}

template <typename T>
static void bn_forward_t(const BNArgs& a, hipStream_t st) {
  if (a.training) bn_stats_t<T>(a, st);
  bn_apply_t<T>(a, st);
}

template <typename T>
static void bn_backward_t(const BNArgs& a, hipStream_t st) {
  const T* x = static_cast<const T*>(a.x);
  const T* dy = static_cast<const T*>(a.dy);
  const T* y = static_cast<const T*>(a.y);
  T* dx = static_cast<T*>(a.dx);
  T* dres = static_cast<T*>(a.dres);
  const int64_t n8 = a.M * a.C / 8;
  int64_t rpb;
  int nb;
  reduce_geometry(a.M, a.C, rpb, nb);
  // relu mask: recompute from x when the forward had no residual (saves reading y)
  const int rmode = !a.relu ? 0 : (a.bits ? 3 : (a.scale ? 2 : 1));
  const float* part = a.partial;
  int rstride = 0;
  if (a.stat_rows) {
    // the kernel that produced dy already reduced (Σdy', Σdy'·(x−mean)) per tile group
    // (bnfuse.hip S2: BN2's sums from the fused BN3 kernel): only fold its rows — in place, as
    // the forward finalize does, up to kColsumDirectMax rows
    const int64_t R = a.stats_rows_n;
    if (R <= kColsumDirectMax) {
      part = a.stat_rows;
      rstride = 2 * a.C;
      nb = (int)R;
    } else {
      nb = colsum_blocks(R);
      const int64_t rows_pb = (R + nb - 1) / nb;
      nb = (int)((R + rows_pb - 1) / rows_pb);
      hipLaunchKernelGGL(k_colsum, dim3(nb), dim3(256), 0, st, a.stat_rows, R, 2 * a.C, rows_pb,
                         a.partial);
    }
  } else {
#define LW_RED(R)                                                                                \
  hipLaunchKernelGGL((k_bn_reduce<T, 1, R, kReduceUnroll>),                                     \
                     dim3(nb, reduce_slices(a.C)), dim3(BNT), 0, st, x, dy, y, a.bits, a.mean, \
                     a.scale, a.shift, a.M, a.C, rpb, a.partial, (const T*)nullptr,      \
                     (const float*)nullptr, (float*)nullptr)
    if (rmode == 0) LW_RED(0); else if (rmode == 1) LW_RED(1); else if (rmode == 2) LW_RED(2);
    else LW_RED(3);
#undef LW_RED
  }
  hipLaunchKernelGGL(k_bn_finalize_bwd, dim3((a.C + 3) / 4), dim3(256), 0, st, part, nb,
                     a.C, a.M, a.gamma, a.mean, a.invstd, a.dgamma, a.dbeta, a.A, a.B, a.Cc,
                     (int)a.training, (int)a.accum_dparams, rstride);
  if (a.coeffs_only) return;
  const dim3 grid(apply_grid(n8, a.C, kApplyBwdGrid)), block(BNT);
#define LW_BWD(R, D)                                                                            \
  hipLaunchKernelGGL((k_bn_bwd_apply<T, R, D>), grid, block, 0, st, x, dy, y, a.bits, a.scale,  \
                     a.shift, a.A, a.B, a.Cc, dx, dres, n8, a.C)
  if (rmode == 3) { if (dres) LW_BWD(3, true); else LW_BWD(3, false); }
  else if (rmode == 1) { if (dres) LW_BWD(1, true); else LW_BWD(1, false); }
  else if (rmode == 2) { if (dres) LW_BWD(2, true); else LW_BWD(2, false); }
  else { if (dres) LW_BWD(0, true); else LW_BWD(0, false); }
#undef LW_BWD
}

// Two BatchNorm+ReLU backwards sharing dy and the ReLU bitmap (bf16, training): a = the first BN
// (x, mean, gamma, ... as in bn_backward), b = the second (its x, mean, invstd, gamma, partial,
// dgamma/dbeta, coefficients and dx); b.dy / b.bits are ignored.
void bn_backward_dual(const BNArgs& a, const BNArgs& b, hipStream_t st) {
  int64_t rpb;
  int nb;
  reduce_geometry(a.M, a.C, rpb, nb, a.M * a.C >= kDualFewBlocksMin ? kDualReduceBlocks : kReduceBlocks);
  const auto* x = static_cast<const uint16_t*>(a.x);
  const auto* x2 = static_cast<const uint16_t*>(b.x);
  const auto* dy = static_cast<const uint16_t*>(a.dy);
  hipLaunchKernelGGL((k_bn_reduce<uint16_t, 1, 3, kReduceUnroll, true>),
                     dim3(nb, reduce_slices(a.C)), dim3(BNT), 0, st, x, dy, (const uint16_t*)nullptr,
                     a.bits, a.mean, (const float*)nullptr, (const float*)nullptr, a.M, a.C, rpb,
                     a.partial, x2, b.mean, b.partial);
  for (const BNArgs* p : {&a, &b})
    hipLaunchKernelGGL(k_bn_finalize_bwd, dim3((p->C + 3) / 4), dim3(256), 0, st, p->partial, nb,
                       p->C, p->M, p->gamma, p->mean, p->invstd, p->dgamma, p->dbeta, p->A, p->B,
                       p->Cc, 1, (int)p->accum_dparams, 0);
  if (a.coeffs_only) return;
  const int64_t n8 = a.M * a.C / 8;
  hipLaunchKernelGGL(k_bn_bwd_apply_dual, dim3(apply_grid(n8, a.C, kApplyBwdGrid)), dim3(BNT), 0, st, x, x2, dy,
                     a.bits, a.A, a.B, a.Cc, b.A, b.B, b.Cc, static_cast<uint16_t*>(a.dx),
                     static_cast<uint16_t*>(b.dx), n8, a.C);
}

void bn_forward(const BNArgs& a, hipStream_t st) {
  if (a.bf16) bn_forward_t<uint16_t>(a, st); else bn_forward_t<float>(a, st);
}
void bn_stats(const BNArgs& a, hipStream_t st) {
  if (a.bf16) bn_stats_t<uint16_t>(a, st); else bn_stats_t<float>(a, st);
}
void bn_apply(const BNArgs& a, hipStream_t st) {
  if (a.bf16) bn_apply_t<uint16_t>(a, st); else bn_apply_t<float>(a, st);
}
void bn_backward(const BNArgs& a, hipStream_t st) {
  if (a.bf16) bn_backward_t<uint16_t>(a, st); else bn_backward_t<float>(a, st);
}

// ------------------------------------------------------------------------------------------
// Fused ResNet stem tail: BatchNorm-apply + ReLU + k×k max-pool (stride s, pad p), NHWC bf16.
// The reference runs conv1 → bn1 → relu → maxpool as separate ops (IMAGENET/training/resnet.py:
// 130-133); here the normalised 112×112 activation is never written: the forward reads the raw
// conv output once and writes the pooled map plus a one-byte window slot per output element; the
// backward routes the pooled gradient straight into the BN backward (reduce + apply), so the
// un-pooled gradient is never materialised either.
// ------------------------------------------------------------------------------------------
struct PoolGeom { int N, H, W, C, Ho, Wo, k, s, p; };

__global__ __launch_bounds__(256) void k_stem_pool_fwd(const uint16_t* __restrict__ x,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift,
                                                       uint16_t* __restrict__ out,
                                                       uint8_t* __restrict__ idx, PoolGeom g) {
  const int G = g.C / 8;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)g.N * g.Ho * g.Wo * G;
  if (t >= total) return;
  // 32-bit index decomposition (the binding guarantees total < 2^31) instead of 64-bit
  // software div/mod; measured neutral on ResNet-50 (stem bwd 0.35 + 0.31 ms either way)
  const uint32_t t32 = (uint32_t)t;
  const int cg = (int)(t32 % (uint32_t)G);
  uint32_t q = t32 / (uint32_t)G;
  const int ow = (int)(q % (uint32_t)g.Wo);
  q /= (uint32_t)g.Wo;
  const int oh = (int)(q % (uint32_t)g.Ho);
  const int n = (int)(q / (uint32_t)g.Ho);
  float sc[8], sh[8], best[8];
  int bi[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = scale[cg * 8 + j]; sh[j] = shift[cg * 8 + j];
    best[j] = -__builtin_huge_valf(); bi[j] = 0;
  }
  for (int kh = 0; kh < g.k; ++kh) {
    const int ih = oh * g.s - g.p + kh;
    if (ih < 0 || ih >= g.H) continue;
    for (int kw = 0; kw < g.k; ++kw) {
      const int iw = ow * g.s - g.p + kw;
      if (iw < 0 || iw >= g.W) continue;
      float v[8];
      V8<uint16_t>::load(x + (((int64_t)n * g.H + ih) * g.W + iw) * g.C + cg * 8, v);
      const int slot = kh * g.k + kw;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a = h2f(f2h(fmaxf(fmaf(v[j], sc[j], sh[j]), 0.f)));
        if (a > best[j]) { best[j] = a; bi[j] = slot; }      // first max wins (PyTorch order)
      }
    }
  }
  const int64_t o = t * 8;
  V8<uint16_t>::store(out + o, best);
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    lo |= (uint32_t)bi[j] << (8 * j);
    hi |= (uint32_t)bi[j + 4] << (8 * j);
  }
  *reinterpret_cast<uint2*>(idx + o) = make_uint2(lo, hi);
}

// Gradient reaching input element (n, ih, iw, 8 channels) through the pool and the ReLU.
__device__ __forceinline__ void stem_dz(const uint16_t* __restrict__ dp,
                                        const uint8_t* __restrict__ idx, const PoolGeom& g, int n,
                                        int ih, int iw, int cg, const float xv[8],
                                        const float sc[8], const float sh[8], float dz[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) dz[j] = 0.f;
  const int oh0 = max(0, (ih + g.p - g.k + g.s) / g.s), oh1 = min(g.Ho - 1, (ih + g.p) / g.s);
  const int ow0 = max(0, (iw + g.p - g.k + g.s) / g.s), ow1 = min(g.Wo - 1, (iw + g.p) / g.s);
  for (int oh = oh0; oh <= oh1; ++oh) {
    const int kh = ih - (oh * g.s - g.p);
    if (kh < 0 || kh >= g.k) continue;
    for (int ow = ow0; ow <= ow1; ++ow) {
      const int kw = iw - (ow * g.s - g.p);
      if (kw < 0 || kw >= g.k) continue;
      const int slot = kh * g.k + kw;
      const int64_t o = (((int64_t)n * g.Ho + oh) * g.Wo + ow) * g.C + cg * 8;
      const uint2 ii = *reinterpret_cast<const uint2*>(idx + o);
      float d[8];
      V8<uint16_t>::load(dp + o, d);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int s8 = (int)(((j < 4 ? ii.x : ii.y) >> (8 * (j & 3))) & 0xffu);
        dz[j] += s8 == slot ? d[j] : 0.f;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) dz[j] = fmaf(xv[j], sc[j], sh[j]) > 0.f ? dz[j] : 0.f;
}

// MODE 0: per-block channel partials of (Σdz, Σdz·(x-mean)) -> [2][C][nb] (fixed order);
// MODE 1: dx = A·dz + B·x + C.
template <int MODE>
__global__ __launch_bounds__(BNT) void k_stem_pool_bwd(const uint16_t* __restrict__ dp,
                                                       const uint8_t* __restrict__ idx,
                                                       const uint16_t* __restrict__ x,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ A,
                                                       const float* __restrict__ B,
                                                       const float* __restrict__ Cc,
                                                       uint16_t* __restrict__ dx,
                                                       float* __restrict__ partial, PoolGeom g,
                                                       int64_t rows_per_block) {
  __shared__ float sa[BNT * 8];
  __shared__ float sb[BNT * 8];
  const int G = g.C / 8;
  const int R = BNT / G;
  const int cg = threadIdx.x % G, r = threadIdx.x / G;
  const bool active = r < R;
  const int64_t M = (int64_t)g.N * g.H * g.W;
  float sc[8], sh[8], mu[8], ca[8], cb[8], cc[8], a[8], b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = active ? cg * 8 + j : 0;
    sc[j] = scale[c]; sh[j] = shift[c];
    mu[j] = MODE == 0 ? mean[c] : 0.f;
    ca[j] = MODE == 1 ? A[c] : 0.f; cb[j] = MODE == 1 ? B[c] : 0.f; cc[j] = MODE == 1 ? Cc[c] : 0.f;
    a[j] = 0.f; b[j] = 0.f;
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(r0 + rows_per_block, M);
  if (active) {
    for (int64_t row = r0 + r; row < r1; row += R) {
      const uint32_t r32 = (uint32_t)row;                  // M < 2^31 (binding check)
      const int iw = (int)(r32 % (uint32_t)g.W);
      const uint32_t q = r32 / (uint32_t)g.W;
      const int ih = (int)(q % (uint32_t)g.H), n = (int)(q / (uint32_t)g.H);
      float xv[8], dz[8];
      V8<uint16_t>::load(x + row * g.C + cg * 8, xv);
      stem_dz(dp, idx, g, n, ih, iw, cg, xv, sc, sh, dz);
      if (MODE == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { a[j] += dz[j]; b[j] += dz[j] * (xv[j] - mu[j]); }
      } else {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = ca[j] * dz[j] + cb[j] * xv[j] + cc[j];
        V8<uint16_t>::store(dx + row * g.C + cg * 8, o);
      }
    }
  }
  if (MODE == 1) return;
  if (active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { sa[r * g.C + cg * 8 + j] = a[j]; sb[r * g.C + cg * 8 + j] = b[j]; }
  }
  __syncthreads();
  const int64_t nb = gridDim.x;
  for (int c = threadIdx.x; c < g.C; c += BNT) {
    float s1 = 0.f, s2 = 0.f;
    for (int qq = 0; qq < R; ++qq) { s1 += sa[qq * g.C + c]; s2 += sb[qq * g.C + c]; }
    partial[(int64_t)c * nb + blockIdx.x] = s1;
    partial[((int64_t)g.C + c) * nb + blockIdx.x] = s2;
  }
}

// 3x3 / stride 2 / pad 1 pool with H == 2*Ho, W == 2*Wo (the ResNet stem): thread (g, r) takes
// the 2x2 input block (2y..2y+1, 2x..2x+1) of output-grid point (y, x) — exactly the pixels
// windows (y|y+1, x|x+1) cover — so every load is issued up front (4 windows' gradients and
// argmax slots, 4 input pixels) with no data-dependent loop, and each window is read by the 4
// blocks that share it (L2 hits) instead of each input pixel walking its windows serially.
// Input row 2y+a is reached by window row y at kh = 1 + a and, for a = 1, by row y+1 at kh = 0.
template <int MODE>
__global__ __launch_bounds__(BNT) void k_stem_pool_bwd_s2(const uint16_t* __restrict__ dp,
                                                          const uint8_t* __restrict__ idx,
                                                          const uint16_t* __restrict__ x,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ shift,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ A,
                                                          const float* __restrict__ B,
                                                          const float* __restrict__ Cc,
                                                          uint16_t* __restrict__ dx,
                                                          float* __restrict__ partial, PoolGeom g,
                                                          int64_t rows_per_block) {
  __shared__ float sa[BNT * 8];
  __shared__ float sb[BNT * 8];
  const int G = g.C / 8;
  const int R = BNT / G;
  const int cg = threadIdx.x % G, r = threadIdx.x / G;
  const bool active = r < R;
  const int64_t P = (int64_t)g.N * g.Ho * g.Wo;          // output-grid points = 2x2 blocks
  float sc[8], sh[8], mu[8], ca[8], cb[8], cc[8], a[8], b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = active ? cg * 8 + j : 0;
    sc[j] = scale[c]; sh[j] = shift[c];
    mu[j] = MODE == 0 ? mean[c] : 0.f;
    ca[j] = MODE == 1 ? A[c] : 0.f; cb[j] = MODE == 1 ? B[c] : 0.f; cc[j] = MODE == 1 ? Cc[c] : 0.f;
    a[j] = 0.f; b[j] = 0.f;
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(r0 + rows_per_block, P);
  if (active) {
    for (int64_t pt = r0 + r; pt < r1; pt += R) {
      const uint32_t p32 = (uint32_t)pt;                   // P < 2^31 (binding check)
      const int xo = (int)(p32 % (uint32_t)g.Wo);
      const uint32_t q = p32 / (uint32_t)g.Wo;
      const int yo = (int)(q % (uint32_t)g.Ho), n = (int)(q / (uint32_t)g.Ho);
      // windows (yo + u, xo + v), u, v in {0, 1}; missing ones (past the grid) contribute 0
      float d[2][2][8];
      uint2 s8[2][2];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v) {
          const bool in = yo + u < g.Ho && xo + v < g.Wo;
          const int64_t o = (((int64_t)n * g.Ho + yo + u) * g.Wo + xo + v) * g.C + cg * 8;
          if (in) {
            V8<uint16_t>::load(dp + o, d[u][v]);
            s8[u][v] = *reinterpret_cast<const uint2*>(idx + o);
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) d[u][v][j] = 0.f;
            s8[u][v] = make_uint2(0xffffffffu, 0xffffffffu);   // slot 255 matches nothing
          }
        }
      float xv[2][2][8];
#pragma unroll
      for (int ay = 0; ay < 2; ++ay)
#pragma unroll
        for (int bx = 0; bx < 2; ++bx)
          V8<uint16_t>::load(x + (((int64_t)n * g.H + 2 * yo + ay) * g.W + 2 * xo + bx) * g.C + cg * 8,
                             xv[ay][bx]);
#pragma unroll
      for (int ay = 0; ay < 2; ++ay)
#pragma unroll
        for (int bx = 0; bx < 2; ++bx) {
          float dz[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float acc = 0.f;
#pragma unroll
            for (int u = 0; u <= ay; ++u)            // window row yo+u reaches row 2yo+ay at kh
#pragma unroll
              for (int v = 0; v <= bx; ++v) {
                const int kh = 1 + ay - 2 * u, kw = 1 + bx - 2 * v;
                const uint32_t w = j < 4 ? s8[u][v].x : s8[u][v].y;
                const int slot = (int)((w >> (8 * (j & 3))) & 0xffu);
                acc += slot == kh * 3 + kw ? d[u][v][j] : 0.f;
              }
            dz[j] = fmaf(xv[ay][bx][j], sc[j], sh[j]) > 0.f ? acc : 0.f;
          }
          if (MODE == 0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) { a[j] += dz[j]; b[j] += dz[j] * (xv[ay][bx][j] - mu[j]); }
          } else {
            float o[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = ca[j] * dz[j] + cb[j] * xv[ay][bx][j] + cc[j];
            V8<uint16_t>::store(dx + (((int64_t)n * g.H + 2 * yo + ay) * g.W + 2 * xo + bx) * g.C + cg * 8, o);
          }
        }
    }
  }
  if (MODE == 1) return;
  if (active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { sa[r * g.C + cg * 8 + j] = a[j]; sb[r * g.C + cg * 8 + j] = b[j]; }
  }
  __syncthreads();
  const int64_t nb = gridDim.x;
  for (int c = threadIdx.x; c < g.C; c += BNT) {
    float s1 = 0.f, s2 = 0.f;
    for (int qq = 0; qq < R; ++qq) { s1 += sa[qq * g.C + c]; s2 += sb[qq * g.C + c]; }
    partial[(int64_t)c * nb + blockIdx.x] = s1;
    partial[((int64_t)g.C + c) * nb + blockIdx.x] = s2;
  }
}

// Reduce pass of the stem backward from the POOLED side. The routed gradient dz is non-zero only
// at each window's argmax, where relu(scale·x + shift) is exactly the stored pooled value p, so
//   Σdz = Σ_{p > 0} d   and   Σdz·(x - mean) = Σ_{p > 0} d·(p - beta) / scale,
// beta = shift + mean·scale (linear in dz, so overlapping windows need no care). The pass reads
// the pooled gradient and the pooled map (2 x N·Ho·Wo·C bf16) instead of the 4x larger conv output
// plus the slot bytes. A channel where that inversion is ill-conditioned reads x at the argmax
// through the slot byte instead: scale == 0 (p constant, x not recoverable), or |beta| large
// against |scale|·sigma = |gamma| — p's bf16 rounding (~2^-9·|beta|) would then become an error of
// up to 2^-9·|beta/gamma| standard deviations in every recovered x - mean, a per-channel bias in
// dgamma. Partials as k_stem_pool_bwd<0>: [2][C][nb].
__global__ __launch_bounds__(BNT) void k_stem_pool_reduce_out(const uint16_t* __restrict__ dp,
                                                              const uint16_t* __restrict__ pooled,
                                                              const uint8_t* __restrict__ idx,
                                                              const uint16_t* __restrict__ x,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ shift,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ invstd,
                                                              float* __restrict__ partial,
                                                              PoolGeom g, int64_t rows_per_block) {
  __shared__ float sa[BNT * 8];
  __shared__ float sb[BNT * 8];
  const int G = g.C / 8;
  const int R = BNT / G;
  const int cg = threadIdx.x % G, r = threadIdx.x / G;
  const bool active = r < R;
  const int64_t P = (int64_t)g.N * g.Ho * g.Wo;
  float sc[8], rs[8], be[8], mu[8], a[8], b[8];
  bool ill[8];
  bool degen = false;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = active ? cg * 8 + j : 0;
    sc[j] = scale[c]; mu[j] = mean[c];
    be[j] = fmaf(mu[j], sc[j], shift[c]);
    // |beta| > 8·|gamma| (gamma = scale / invstd): recover x - mean by gathering x instead
    ill[j] = sc[j] == 0.f || fabsf(be[j]) * invstd[c] > 8.f * fabsf(sc[j]);
    rs[j] = ill[j] ? 0.f : 1.f / sc[j];
    degen |= ill[j];
    a[j] = 0.f; b[j] = 0.f;
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(r0 + rows_per_block, P);
  constexpr int U = 4;                                // rows per iteration, loads all in flight
  if (active) {
    for (int64_t pt0 = r0 + r; pt0 < r1; pt0 += U * R) {
      float d[U][8], p[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t pt = pt0 + u * R;
        if (pt < r1) {
          V8<uint16_t>::load(dp + pt * g.C + cg * 8, d[u]);
          V8<uint16_t>::load(pooled + pt * g.C + cg * 8, p[u]);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) { d[u][j] = 0.f; p[u][j] = 0.f; }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float dz = p[u][j] > 0.f ? d[u][j] : 0.f;
          a[j] += dz;
          b[j] += dz * ((p[u][j] - be[j]) * rs[j]);
        }
      if (degen) {                                   // rare: gather x at the argmax
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t pt = pt0 + u * R;
          if (pt >= r1) continue;
          const int64_t o = pt * g.C + cg * 8;
          const uint32_t p32 = (uint32_t)pt;
          const int ow = (int)(p32 % (uint32_t)g.Wo);
          const uint32_t q = p32 / (uint32_t)g.Wo;
          const int oh = (int)(q % (uint32_t)g.Ho), n = (int)(q / (uint32_t)g.Ho);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            if (!ill[j] || !(p[u][j] > 0.f)) continue;
            const int slot = idx[o + j];
            const int ih = oh * g.s - g.p + slot / g.k, iw = ow * g.s - g.p + slot % g.k;
            const float xv = h2f(x[(((int64_t)n * g.H + ih) * g.W + iw) * g.C + cg * 8 + j]);
            b[j] += d[u][j] * (xv - mu[j]);
          }
        }
      }
    }
  }
  if (active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { sa[r * g.C + cg * 8 + j] = a[j]; sb[r * g.C + cg * 8 + j] = b[j]; }
  }
  __syncthreads();
  const int64_t nb = gridDim.x;
  for (int c = threadIdx.x; c < g.C; c += BNT) {
    float s1 = 0.f, s2 = 0.f;
    for (int qq = 0; qq < R; ++qq) { s1 += sa[qq * g.C + c]; s2 += sb[qq * g.C + c]; }
    partial[(int64_t)c * nb + blockIdx.x] = s1;
    partial[((int64_t)g.C + c) * nb + blockIdx.x] = s2;
  }
}

void stem_pool_fwd(const StemArgs& a, hipStream_t st) {
  const PoolGeom g{a.N, a.H, a.W, a.C, a.Ho, a.Wo, a.k, a.s, a.p};
  const int64_t total = (int64_t)a.N * a.Ho * a.Wo * (a.C / 8);
  hipLaunchKernelGGL(k_stem_pool_fwd, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     static_cast<const uint16_t*>(a.x), a.scale, a.shift,
                     static_cast<uint16_t*>(a.out), a.idx, g);
}

// Apply passes: the reduce geometry (~512 blocks walking ~50 rows each). One row per thread
// (a grid of ~25k blocks) measured slower: stem pool backward +50 us, CIFAR ResNet-9 -15 %
// (profiles/r3s2/stem_ab.txt).
static void pool_apply_geometry(int64_t rows, int C, int64_t& rpb, int& nb) {
  reduce_geometry(rows, C, rpb, nb);
}

// The stride-2 2x2-block apply (one output grid point's four input pixels per row): ~4k
// workgroups, 229 vs 267 us for the stem's 112 -> 56 backward at 512 (profiles/r6/
// bn_stream_probe2.txt; the statistics pass stays at the reduce geometry, 39 us there)
constexpr int64_t kPoolS2ApplyBlocks = 4096;
static void pool_s2_apply_geometry(int64_t rows, int C, int64_t& rpb, int& nb) {
  reduce_geometry(rows, C, rpb, nb, kPoolS2ApplyBlocks);
}

// Max-pool of a post-ReLU map without a BatchNorm (VGG / AlexNet conv+ReLU -> MaxPool2d): the
// forward is k_stem_pool_fwd with scale 1 / shift 0 (relu(v) == v there), the backward only the
// apply pass with (A, B, C) = (1, 0, 0): dx = the routed pooled gradient masked by [x > 0], i.e.
// the max-pool AND the preceding ReLU backward in one kernel. a.A / a.B / a.Cc / a.scale / a.shift
// must hold those constants (the binding fills them).
// [ones][zeros], kPoolIdC each, initialised at module load (no kernel, graph-capture safe)
struct PoolIdentity { float v[2 * kPoolIdC]; };
constexpr PoolIdentity make_pool_identity() {
  PoolIdentity p{};
  for (int i = 0; i < kPoolIdC; ++i) p.v[i] = 1.f;
  return p;
}
__device__ PoolIdentity kPoolIdentity = make_pool_identity();

const float* pool_identity_consts() {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(kPoolIdentity)) != hipSuccess) return nullptr;
  return static_cast<const float*>(p);
}

void relu_pool_bwd(const StemArgs& a, hipStream_t st) {
  const PoolGeom g{a.N, a.H, a.W, a.C, a.Ho, a.Wo, a.k, a.s, a.p};
  const auto* dp = static_cast<const uint16_t*>(a.dp);
  const auto* x = static_cast<const uint16_t*>(a.x);
  if (a.k == 3 && a.s == 2 && a.p == 1 && a.H == 2 * a.Ho && a.W == 2 * a.Wo) {
    const int64_t P = (int64_t)a.N * a.Ho * a.Wo;
    int64_t rpb;
    int nb;
    pool_s2_apply_geometry(P, a.C, rpb, nb);
    hipLaunchKernelGGL((k_stem_pool_bwd_s2<1>), dim3(nb), dim3(BNT), 0, st, dp, a.idx, x, a.scale,
                       a.shift, a.mean, a.A, a.B, a.Cc, static_cast<uint16_t*>(a.dx),
                       (float*)nullptr, g, rpb);
    return;
  }
  const int64_t M = (int64_t)a.N * a.H * a.W;
  int64_t rpb;
  int nb;
  pool_apply_geometry(M, a.C, rpb, nb);
  hipLaunchKernelGGL((k_stem_pool_bwd<1>), dim3(nb), dim3(BNT), 0, st, dp, a.idx, x, a.scale,
                     a.shift, a.mean, a.A, a.B, a.Cc, static_cast<uint16_t*>(a.dx),
                     (float*)nullptr, g, rpb);
}

void stem_pool_bwd(const StemArgs& a, hipStream_t st) {
  const PoolGeom g{a.N, a.H, a.W, a.C, a.Ho, a.Wo, a.k, a.s, a.p};
  const int64_t M = (int64_t)a.N * a.H * a.W;
  int64_t rpb;
  int nb;
  reduce_geometry(M, a.C, rpb, nb);
  const auto* dp = static_cast<const uint16_t*>(a.dp);
  const auto* x = static_cast<const uint16_t*>(a.x);
  const int64_t P = (int64_t)a.N * a.Ho * a.Wo;
  int64_t rpb2;
  int nb2;
  reduce_geometry(P, a.C, rpb2, nb2);
  if (a.pooled) {   // statistics from the pooled side (any geometry); partials over nb2 blocks
    hipLaunchKernelGGL(k_stem_pool_reduce_out, dim3(nb2), dim3(BNT), 0, st, dp,
                       static_cast<const uint16_t*>(a.pooled), a.idx, x, a.scale, a.shift, a.mean,
                       a.invstd, a.partial, g, rpb2);
    hipLaunchKernelGGL(k_bn_finalize_bwd, dim3((a.C + 3) / 4), dim3(256), 0, st, a.partial, nb2,
                       a.C, M, a.gamma, a.mean, a.invstd, a.dgamma, a.dbeta, a.A, a.B, a.Cc, 1,
                       (int)a.accum_dparams, 0);
    if (a.coeffs_only) return;
  }
  if (a.k == 3 && a.s == 2 && a.p == 1 && a.H == 2 * a.Ho && a.W == 2 * a.Wo) {
    // 2x2-block form over the output grid (same partial layout: nb blocks of the grid points)
    if (!a.pooled) {
      hipLaunchKernelGGL((k_stem_pool_bwd_s2<0>), dim3(nb2), dim3(BNT), 0, st, dp, a.idx, x,
                         a.scale, a.shift, a.mean, (const float*)nullptr, (const float*)nullptr,
                         (const float*)nullptr, (uint16_t*)nullptr, a.partial, g, rpb2);
      hipLaunchKernelGGL(k_bn_finalize_bwd, dim3((a.C + 3) / 4), dim3(256), 0, st, a.partial,
                         nb2, a.C, M, a.gamma, a.mean, a.invstd, a.dgamma, a.dbeta, a.A, a.B, a.Cc,
                         1, (int)a.accum_dparams, 0);
    }
    int64_t rpa;
    int nba;
    pool_s2_apply_geometry(P, a.C, rpa, nba);
    hipLaunchKernelGGL((k_stem_pool_bwd_s2<1>), dim3(nba), dim3(BNT), 0, st, dp, a.idx, x, a.scale,
                       a.shift, a.mean, a.A, a.B, a.Cc, static_cast<uint16_t*>(a.dx),
                       (float*)nullptr, g, rpa);
    return;
  }
  if (!a.pooled) {
    hipLaunchKernelGGL((k_stem_pool_bwd<0>), dim3(nb), dim3(BNT), 0, st, dp, a.idx, x, a.scale,
                       a.shift, a.mean, (const float*)nullptr, (const float*)nullptr,
                       (const float*)nullptr, (uint16_t*)nullptr, a.partial, g, rpb);
    hipLaunchKernelGGL(k_bn_finalize_bwd, dim3((a.C + 3) / 4), dim3(256), 0, st, a.partial, nb,
                       a.C, M, a.gamma, a.mean, a.invstd, a.dgamma, a.dbeta, a.A, a.B, a.Cc, 1,
                       (int)a.accum_dparams, 0);
  }
  int64_t rpa;
  int nba;
  pool_apply_geometry(M, a.C, rpa, nba);
  hipLaunchKernelGGL((k_stem_pool_bwd<1>), dim3(nba), dim3(BNT), 0, st, dp, a.idx, x, a.scale,
                     a.shift, a.mean, a.A, a.B, a.Cc, static_cast<uint16_t*>(a.dx),
                     (float*)nullptr, g, rpa);
}

}  // namespace lw
