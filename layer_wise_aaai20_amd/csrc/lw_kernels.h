// Host-visible launcher API of the layer_wise_aaai20_amd HIP kernels (gfx950).
// Kernels take raw device pointers + a hipStream_t so they can be driven from the torch op
// bindings (bindings.cpp) or from the native C++ runtime alike.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace lw {

constexpr int kLargeEPB = 8192;    // elements per workgroup in multi-block passes
constexpr int kWriteSub = 4;          // sub-tasks per task in the fused chain's count / write
constexpr int kSmallMax = 4096;    // segments up to this size use the single-workgroup path
constexpr int kUnpackChunk = 4096; // elements per workgroup in the pair unpack
constexpr int kMaxWorld = 64;

enum KeyMode { KM_TOPK = 0, KM_RANDK = 1, KM_THRESH = 2 };
enum OutMode { OUT_PAIRS = 0, OUT_VALIDX = 1 };
enum QuantMode { Q_TERN = 0, Q_QS8 = 1, Q_QS9 = 2, Q_QS16 = 3 };

__host__ __device__ constexpr int64_t hdr_words(int64_t nseg) { return (nseg + 3) / 4 * 4; }

struct SelState {
  uint32_t prefix;   // radix digits chosen so far
  uint32_t m;        // rank of the wanted key inside the current prefix bucket (1-based)
  uint32_t tkey;     // final threshold key
  uint32_t quota;    // how many keys == tkey are emitted
  uint32_t cnt_gt;   // keys > tkey in the segment
  uint32_t total;    // emitted elements
  uint32_t cap;      // payload slots of the segment
  uint32_t pad;
  // the fused radix chain (compress.hip k_hist_sel / k_count_sel): the digit state after passes
  // 0 and 1, published by one workgroup for the next launch in fields that launch does not write
  uint32_t p0, m0, p1, m1;
};

// Momentum correction fused into the first pass of the Top-K chain (layer-wise buckets;
// compress.hip mc_step): u = mc·u + (g + wmul·wd_s·p) per element, and the compressor sees u.
// u == nullptr: no fused prologue (parallel/engine.py runs optim.hip k_mc_prep instead, or none).
struct McArgs {
  float* u;                    // velocity (the bucket's layout)
  const float* p;              // parameters (nullptr: no weight decay)
  const float* wd;             // [S] weight decay per codec segment (nullptr: none)
  float mc, wmul;
};

struct SelectArgs {
  float* g;                    // bucket base (fp32 gradient arena slice)
  float* ef;                   // error-feedback residual (same layout) or nullptr
  const int64_t* seg_off;      // [S+1] element offsets within the bucket
  const int32_t* seg_n;        // [S]   true element counts
  const int32_t* keep;         // [S]   m_s (Top-K / Random-K)
  const int64_t* cap_off;      // [S+1] payload slot offsets
  const int32_t* small_segs;   // [n_small]
  const int32_t* large_segs;   // [n_large]
  const int2* tasks;           // [n_tasks] (large index, begin)
  const int32_t* task_lo;      // [n_large+1]
  int n_small, n_large, n_tasks;
  int max_seg_tasks;           // most tasks of one large segment (0: unknown)
  // scratch
  uint32_t* hist;              // [n_large*4096]
  SelState* st_small;          // [n_small]
  SelState* st_large;          // [n_large]
  uint2* cnt;                  // [n_tasks]
  uint2* pre;                  // [n_tasks]
  // outputs
  int2* pairs;                 // OUT_PAIRS: [cap_total] (index, float bits)
  float* vals;                 // OUT_VALIDX
  int32_t* idx_out;            // OUT_VALIDX
  // rng
  uint32_t gid_base, step, seed0, seed1;
  const uint32_t* step_ptr;    // optional device step counter (overrides `step`; HIP graphs)
  // optional momentum-correction velocity (same layout as g): zeroed at every coordinate that was
  // sent, in segments that were not sent whole (those keep ordinary momentum)
  float* mom;
  McArgs mcx;                  // fused momentum-correction prologue (mcx.u == nullptr: none)
  // optional device counter: elements the reference rule would send that did not fit the
  // payload (Top-K ties beyond the tie slack; threshold hits beyond a fixed sparse capacity)
  unsigned long long* overflow;
};

struct QuantArgs {
  float* g;
  float* ef;
  const int64_t* seg_off;
  const int32_t* seg_n;
  const int32_t* segs;         // all segments (large path)
  const int2* tasks;
  const int32_t* task_lo;
  const int64_t* rec_off;      // [S+1] group-record offsets (32 elements per group)
  int nseg, n_tasks, qstates;
  float* scale;                // [S] abs-max (TernGrad) or L2 norm (QSGD)
  uint32_t* payload;           // this rank's send buffer
  uint32_t gid_base, step, tag, seed0, seed1;
  const uint32_t* step_ptr;    // optional device step counter (overrides `step`; HIP graphs)
};

void select_compress(const SelectArgs& a, int km, int out, bool ef, hipStream_t st,
                     bool staged = false);
// entire-model staging (compress.hip): pass 0 over tasks [t_lo, t_hi) while backward runs
void select_stage(const SelectArgs& a, int km, bool ef, int t_lo, int t_hi, bool zero,
                  hipStream_t st);
void thresh_count(const SelectArgs& a, float V, int adaptive, bool ef, float* segmax,
                  float2* partial, int32_t* count_out, hipStream_t st);
void thresh_write(const SelectArgs& a, bool ef, hipStream_t st);
void thresh_dense(const SelectArgs& a, float V, int adaptive, bool ef, float* segmax,
                  float2* partial, hipStream_t st);
void unpack_pairs(const int2* gathered, int64_t cap_total, int ws, float* g, const int64_t* seg_off,
                  const int32_t* seg_n, const int64_t* cap_off, const int2* utasks, int n_utasks,
                  hipStream_t st);
void unpack_validx(const float* vals, const int32_t* idx, const int32_t* slot_seg, int64_t nslots,
                   int ws, float* g, const int64_t* seg_off, hipStream_t st);
void seg_reduce(const QuantArgs& a, bool ef_add, int what, float* out, float2* partial,
                hipStream_t st, bool staged = false);
void quant_stage(const QuantArgs& a, bool ef_add, int t_lo, int t_hi, float2* partial,
                 hipStream_t st);
void quantize(const QuantArgs& a, int q, bool ef, hipStream_t st);
void dequantize(const QuantArgs& a, int q, const uint32_t* gathered, int64_t words_per_rank, int ws,
                hipStream_t st);
// quantised reduce-scatter wire (compress.hip): one shard's rank-ordered dequantise-and-average
// into a bf16 bucket image, and that image expanded into the fp32 gradient
void dequantize_shard(int q, const uint32_t* recv, int64_t wpr, int ws, int hdr, const int4* gtab,
                      int64_t g0, int64_t ng, int qstates, uint16_t* out, int64_t n_out,
                      hipStream_t st);
void bf16_expand(const uint16_t* in, float* out, int64_t n, hipStream_t st);
// simulated xGMI transfer time: nwg workgroups busy for `us` microseconds (loopback wire model)
void wire_wait(double us, int nwg, hipStream_t st);

// optimizer (optim.hip)
struct SgdArgs {
  float* p;                    // flat param arena
  const float* g;              // flat grad arena
  float* buf;                  // flat momentum arena
  const int64_t* seg_off;
  const int32_t* seg_n;
  const int32_t* segs;
  const int2* tasks;
  const float* seg_wd;         // [S] weight decay per segment
  int n_tasks;
  float lr, momentum, dampening, grad_scale;
  int nesterov, first_step;
  const float* hyper;          // optional device [lr, grad_scale] (overrides the scalars)
  uint16_t* pb;                // optional bf16 mirror of p (same layout), written in the same pass
};
void sgd_step(const SgdArgs& a, hipStream_t st);
// decode of a Top-K bucket fused with the SGD step of its elements (compress.hip k_unpack_sgd;
// ftasks: {codec segment, chunk begin, chunk end, parameter}; `a` points at the bucket: p / buf /
// pb / seg_wd offset to its first element / parameter, g unused)
void unpack_pairs_sgd(const int2* gathered, int64_t cap_total, int ws, const int64_t* seg_off,
                      const int64_t* cap_off, const int4* ftasks, int n_ftasks, const SgdArgs& a,
                      hipStream_t st);
// momentum correction (optim.hip): the compressor prologue g' = g + wmul·wd·p, u = mc·u + g',
// g = u over a bucket's arena segments (p / seg_wd null: no weight decay), and the velocity masking
// u = 0 where e == 0 for codecs without a selection
void mc_prep(float* g, float* u, const float* p, const int64_t* seg_off, const int32_t* seg_n,
             const int32_t* segs, const int2* tasks, int n_tasks, const float* seg_wd, float mc,
             float wmul, hipStream_t st);
void mc_mask(float* u, const float* e, int64_t n, hipStream_t st);
void step_bump(int64_t* c, hipStream_t st);

// fused BatchNorm (+add) (+ReLU), NHWC (bn.hip)
struct BNArgs {
  const void* x;        // [M, C] bf16 or fp32
  const void* res;      // residual (forward) or nullptr
  void* y;              // forward output; backward: saved output for the ReLU mask (or nullptr)
  const void* dy;
  void* dx;
  void* dres;           // backward: gradient w.r.t. the residual input (or nullptr)
  int64_t M;
  int C;
  bool bf16, training, relu;
  float eps, momentum;
  const float* gamma;   // may be nullptr (affine=False)
  const float* beta;
  float* rmean;         // running stats (nullptr: not tracked)
  float* rvar;
  float* mean;          // [C] batch mean (saved)
  float* invstd;        // [C]
  float* scale;         // [C] forward scratch
  float* shift;         // [C]
  float* partial;       // [nblocks][2C]
  float* dgamma;
  float* dbeta;
  float* A;             // [C] backward coefficients
  float* B;
  float* Cc;
  const float* res_scale;  // forward: residual through its own BN affine (or nullptr)
  const float* res_shift;
  int stats_blocks;        // bn_stats: >0 = partial sums already in `partial` ([2C][nb])
  const float* stat_rows;  // bn_stats: per-M-tile rows [R][2C] from a GEMM epilogue (or nullptr)
  int64_t stats_rows_n;    // R (bn_stats; bn_backward: precomputed (Σdy', Σdy'(x−mean)) rows from
                           // a GEMM's EPI_BSTATS epilogue replace the reduce pass)
  uint8_t* bits;           // ReLU bitmap, 1 bit/element: written by the forward apply, read back
                           // by the backward instead of the saved output (or nullptr)
  bool accum_dparams;      // backward: dgamma/dbeta += (into the gradient arena) instead of =
  bool coeffs_only;        // backward: reduce + finalize only (dx formed by a fused consumer)
};
int bn_reduce_blocks(int64_t M, int C);
int colsum_blocks(int64_t rows);     // blocks folding R GEMM-epilogue statistics rows
void bn_stats(const BNArgs& a, hipStream_t st);
void bn_apply(const BNArgs& a, hipStream_t st);
void bn_forward(const BNArgs& a, hipStream_t st);
void bn_backward(const BNArgs& a, hipStream_t st);
// two BN+ReLU backwards sharing dy and the ReLU bitmap (a bottleneck's BN3 and downsample BN)
void bn_backward_dual(const BNArgs& a, const BNArgs& b, hipStream_t st);
// BN3 backward apply fused with dW3 += dc3ᵀ·a2 and da2 = dc3·W3 (bnfuse.hip): (C, Ci) = (256, 64)
// or (512, 128); slab [bn3_bwd_dgemm_slabs(M, C, Ci)][C][Ci] fp32 partials of dW3 (summed by
// splitk_reduce; with a single slab and acc_out the kernel adds into slab = the destination).
// With x2 (the downsample block: its shortcut BN's input, same dy and bitmap) also
// dx2 = A2·(dy·bit) + B2·x2 + C2 into dx2 [M][C]. With st2: BN2's backward sums
// (Σd, Σd·(c2 − mean2)), d = da2·[c2·ss2 + ss2[Ci..] > 0], one row per slab: st2 [slabs][2][Ci].
// a2c: `a2` is c2 and the kernel forms relu(c2·ss2 + ss2[Ci..]) itself (ss2 required).
// BN1 backward apply fused with dW1 += dc1ᵀ·x and dx = dc1·W1 + dy·bit3 (bnfuse.hip), for a
// bottleneck without downsample: (Wd, Cin) = (64, 256) or (128, 512); the ReLU mask from c1 via
// the forward affine (fs, fh); w1t = W1ᵀ [Cin][Wd]; slab [bn1_bwd_dgemm_slabs][Wd][Cin]
bool bn1_bwd_dgemm_ok(int64_t M, int Wd, int Cin);
int bn1_bwd_dgemm_slabs(int64_t M, int Wd, int Cin);
void bn1_bwd_dgemm(const uint16_t* da1, const uint16_t* c1, const float* fs, const float* fh,
                   const float* A, const float* B, const float* Cc, const uint16_t* w1t,
                   const uint16_t* x, const uint16_t* dy, const uint8_t* bits, uint16_t* dx,
                   float* slab, int64_t M, int Wd, int Cin, bool acc_out, hipStream_t st);
bool bn3_bwd_dgemm_ok(int64_t M, int C, int Ci);
int bn3_bwd_dgemm_slabs(int64_t M, int C, int Ci);
void bn3_bwd_dgemm(const uint16_t* dr, const uint16_t* c3, const uint8_t* bits, const float* A,
                   const float* B, const float* Cc, const uint16_t* w3t, const uint16_t* a2,
                   uint16_t* da2, float* slab, int64_t M, int C, int Ci, hipStream_t st,
                   const uint16_t* x2 = nullptr, const float* A2 = nullptr,
                   const float* B2 = nullptr, const float* C2 = nullptr, uint16_t* dx2 = nullptr,
                   bool acc_out = false, const uint16_t* c2 = nullptr, const float* ss2 = nullptr,
                   const float* mean2 = nullptr, float* st2 = nullptr, bool a2c = false);

// fused stem: BN-apply + ReLU + max-pool (bn.hip), bf16 NHWC
struct StemArgs {
  const void* x;          // conv output [N, H, W, C]
  const float* scale;     // BN scale/shift (forward coefficients)
  const float* shift;
  void* out;              // pooled [N, Ho, Wo, C]
  uint8_t* idx;           // window slot of the max, per pooled element
  const void* dp;         // backward: gradient of the pooled output
  void* dx;               // backward: gradient of the conv output
  const float* gamma;
  const float* mean;
  const float* invstd;
  float* partial;         // [2][C][nb]
  float* dgamma;
  float* dbeta;
  float* A;
  float* B;
  float* Cc;
  const void* pooled;     // backward: the forward's pooled map (statistics from the pooled side)
  int N, H, W, C, Ho, Wo, k, s, p;
  bool accum_dparams;
  bool coeffs_only;       // backward: statistics + finalize only (dx formed by a fused consumer)
};
void stem_pool_fwd(const StemArgs& a, hipStream_t st);
void stem_pool_bwd(const StemArgs& a, hipStream_t st);
void relu_pool_bwd(const StemArgs& a, hipStream_t st);   // pool + ReLU backward, no BN
// the stem's pool/BN backward apply fused with the 7x7/2 conv's weight gradient (stemfuse.hip):
// conv output C = 64 at 112x112 from a 224x224 4-channel image, 3x3/2/1 pool; slab
// [stem_bwd_wgrad_blocks][64][224] fp32 partials of dW [co][r][s 0..7][ci 0..3]
bool stem_bwd_wgrad_ok(int C, int H, int W, int Ho, int Wo, int Hin, int Win);
int stem_bwd_wgrad_blocks(int N, int Ho);
void stem_bwd_wgrad(const uint16_t* dp, const uint8_t* idx, const uint16_t* c, const float* scale,
                    const float* shift, const float* A, const float* B, const float* Cc,
                    const uint16_t* x4, float* slab, int N, int Ho, int Wo, int Hin, int Win,
                    hipStream_t st);
// kPoolIdC ones followed by kPoolIdC zeros in device memory (current device): the identity BN
// constants of a plain ReLU max-pool, so a pool call needs no per-call fill kernels
constexpr int kPoolIdC = 2048;
const float* pool_identity_consts();

// bf16 MFMA GEMM with fused epilogue (gemm.hip)
struct GemmArgs {
  const uint16_t* A;  // bf16
  int64_t lda;
  bool a_kcontig;     // A(m,k) = A[m*lda+k] (true) or A[k*lda+m] (false)
  const uint16_t* B;
  int64_t ldb;
  bool b_kcontig;     // B(k,n) = B[n*ldb+k] (true) or B[k*ldb+n] (false)
  void* C;            // [M, ldc] row-major, bf16 or fp32
  int64_t ldc;
  bool out_bf16;
  const float* bias;  // [N] or nullptr
  int relu;
  int M, N, K;
  int splits;         // split-K factor (>1 needs `partial`)
  float* partial;     // [splits][M][N] fp32
  int tile;           // GemmTile, 0 = heuristic
  float* stats;       // optional [2][N][tiles_m] per-column Σv, Σv² (no split-K)
  const float* pro_scale;  // optional prologue relu(v*scale+shift): per-k of a K-contiguous A
  const float* pro_shift;  // (pro_on_a) or per-n of an N-contiguous B
  bool pro_on_a;
  const uint16_t* addend;  // optional bf16 [M][ldc] added to a bf16 output (dgrad + residual grad)
  const uint8_t* add_bits; // optional ReLU bitmap masking the addend (ldc == N)
  bool accumulate;         // fp32 output: C += result (weight gradients into the zeroed arena)
  uint32_t a_bytes, b_bytes;  // operand extents (< 2 GiB): the buffer loads' range check
  // backward BatchNorm statistics of the bf16 output (EPI_BSTATS, with `stats`): the output is the
  // gradient dy reaching a BN+ReLU whose input was bst_x ([rows][ldc], ldc == N); per M-tile row
  // (Σ dy', Σ dy'·(x − mean)) with dy' = dy·mask, mask from bst_bits (ReLU bitmap of the BN's
  // output) or x*scale+shift > 0 (bst_scale/bst_shift) — the reduce pass of that BN's backward
  const uint16_t* bst_x;
  const float* bst_mean;
  const float* bst_scale;
  const float* bst_shift;
  const uint8_t* bst_bits;
};
enum GemmTile { GEMM_AUTO = 0, GEMM_T128x128x32 = 1, GEMM_T128x128x64 = 2, GEMM_T256x64x32 = 3,
                GEMM_T64x256x32 = 4, GEMM_T256x64x64 = 5,
                GEMM_T64x64x64 = 6,
                // streaming kernel (persistent, B panel resident in LDS, A straight to registers),
                // output-panel width 64 / 128 / 256; K must be 64, 128 or 256
                GEMM_S64 = 11, GEMM_S128 = 12, GEMM_S256 = 13,
                // 256x256 / 256x128 x64 tiles, 8 waves, LDS-DMA kept in flight across barriers
                // (gemm_big.hip): K-/K-, K-/N- or M-/N-contiguous operands, column statistics (one
                // row per 128 rows), split-K slabs; no prologue / addend
                GEMM_B256 = 21, GEMM_B256x128 = 22,
                // the same tiles as a persistent kernel (one workgroup per CU walking tiles, the
                // next tile's first K-tiles loaded during this tile's epilogue): K-contiguous A/B,
                // bf16 output (+ statistics rows, + masked addend), K > 64
                GEMM_P256 = 23, GEMM_P256x128 = 24,
                // the tiles 1..6 on v_mfma_f32_32x32x16 (tile id + 40, gemm_core.h k_gemm MF = 32)
                GEMM_M32 = 40 };
inline bool gemm_is_mf32(int t) { return t > GEMM_M32 && t <= GEMM_M32 + 6; }
inline int gemm_base_tile(int t) { return gemm_is_mf32(t) ? t - GEMM_M32 : t; }
void gemm_bf16(const GemmArgs& g, hipStream_t st);
int gemm_pick_tile(const GemmArgs& g);
int gemm_tiles_m(const GemmArgs& g);
int gemm_splits_used(const GemmArgs& g);
bool gemm_stream_ok(const GemmArgs& g);
// [class][jr][js][Co][C] slabs of a channels_last weight (conv.hip k_pack_dgrad_nkc), C % 8 == 0
void pack_dgrad_nkc(const uint16_t* w, uint16_t* out, int Co, int C, int R, int S, int sh, int sw,
                    int nclass, const int* r0, const int* s0, const int* TR, const int* TS,
                    hipStream_t st);
void pack_dgrad_kc(const uint16_t* w, uint16_t* out, int Co, int C, int R, int S, int sh, int sw,
                   int nclass, const int* r0, const int* s0, const int* TR, const int* TS,
                   int kmax, hipStream_t st);
bool gemm_big_ok(const GemmArgs& g);
bool gemm_bigp_ok(const GemmArgs& g);
void splitk_reduce(const GemmArgs& g, int splits, hipStream_t st);   // fixed-order slab reduce
// deferred reduces (gemm.hip): while on, fp32 split-K outputs without bias / ReLU / addend are
// queued; splitk_take_deferred reports (and clears) whether the last splitk_reduce was queued;
// splitk_flush reduces every queued one in one launch per 24 and returns how many there were
void splitk_set_defer(bool on);
bool splitk_take_deferred();
int splitk_flush(hipStream_t st);
int splitk_discard();            // drop the queue (and its slabs) without launching anything
int splitk_pending();
void gemm_tile_shape(int tile, int& bm, int& bn, int& bk);
int stats_rows_bm(int tile);      // rows of C per column-statistics row of a tile
int gemm_k_per_split(int K, int splits, int bk);

// implicit-GEMM convolution, NHWC bf16 (conv.hip). The GEMM view of each pass:
//   forward  y[pix][co]  = Σ_(tap,ci) X[gather(pix, tap)][ci] · W[co][tap][ci]      A-gather
//   dgrad    dx[pix][ci] = Σ_(tap,co) dY[gather(pix, tap)][co] · Wt[tap][co][ci]    A-gather,
//            per stride-parity class (stride 2: 4 classes, each a stride-1 problem)
//   wgrad    dW[co][tap][ci] = Σ_pix dY[pix][co] · X[gather(pix, tap)][ci]        B-gather
// `g` carries the plain GEMM part (operands, output, epilogue, prologue, split-K), `cv` the
// gather geometry; `mode` is CV_A / CV_A4 / CV_B / CV_B4 of gemm_core.h.
// gather modes: row (A) gather C % 8 / C == 4, column (B) gather C % 8 / C == 4
enum ConvMode { CV_NONE = 0, CV_A = 1, CV_A4 = 2, CV_B = 3, CV_B4 = 4 };
struct ConvGeomHost {
  int Hin, Win, C, sh, sw, dh, dw, Hout, Wout, osy, osx, nclass;
  int TR[4], TS[4], oh[4], ow[4], Hg[4], Wg[4], py[4], px[4], M[4], K[4];
  int64_t b_off[4];
};
void conv_gemm(const GemmArgs& g, const ConvGeomHost& cv, int mode, hipStream_t st);
int conv_splits_used(const GemmArgs& g);
bool conv_tile_ok(int mode, int tile);
// the 256x256 / 256x128 big tiles (GEMM_B256*) on a row-gather conv: one class, identity row
// map, C % 64 == 0, K-contiguous weight, no prologue / addend / backward statistics
bool conv_big_ok(const GemmArgs& g, const ConvGeomHost& h);
// direct 7x7/2 stem convolution from an LDS patch (conv.hip): 4-channel NHWC image, the packed
// [64][7*8*4] weight, bf16 NHWC output + one column-statistics row per 4 output rows
int cu_count();                       // compute units of the current device (cached)
int stem_conv7_blocks(int N, int Ho);  // workgroups (= statistics rows) of stem_conv7
bool stem_conv7_ok(int C, int Co, int R, int S, int sh, int sw, int ph, int pw, int H, int W,
                   int Ho, int Wo);
void stem_conv7(const uint16_t* x, const uint16_t* w, uint16_t* y, float* stats, int N, int H,
                int W, int Ho, int Wo, hipStream_t st);
// tap-reuse 3x3 / stride-1 / pad-1 convolution (conv3tap.hip): x NHWC [N*H*W][C] bf16, w the
// K-contiguous [Co][9C] operand ((r, s, ci) order); stats (optional) [tiles_m][2][Co]
bool conv3_tap_ok(int C, int Co, int H, int W);
int conv3_tap_tiles_m(int N, int H, int W);
void conv3_tap(const uint16_t* x, const uint16_t* w, uint16_t* y, float* stats, int N, int H,
               int W, int C, int Co, hipStream_t st);
// its weight gradient: fp32 dW [Co][3][3][C] (= out, accumulated when `accumulate`), `part` a
// [splits][Co][9][C] fp32 workspace (splits: conv3_tap_wgrad_splits)
int conv3_tap_wgrad_splits(int N, int H, int W, int C, int Co);
void conv3_tap_wgrad(const uint16_t* dy, const uint16_t* x, float* part, float* out, int N,
                     int H, int W, int C, int Co, int accumulate, hipStream_t st);

// model-path elementwise (nn.hip)
void normalize_u8(const uint8_t* in, void* out, int64_t nbytes, const float mean[3],
                  const float stdv[3], bool bf16, hipStream_t st);
void launch_invalid_config_for_test(hipStream_t st);
// bounded busy kernel (<= 30 s) for the communicator-watchdog test (nn.hip)
void spin_for_test(double ms, hipStream_t st);
// global average pool of NHWC bf16 [N, HW, C] (C % 8 == 0): forward to [N, C] bf16, backward
// from [N, C] bf16/fp32 to the channels_last [N, HW, C] bf16 gradient (nn.hip)
void gap_fwd(const uint16_t* x, uint16_t* y, int N, int HW, int C, hipStream_t st);
// out[i] = Σ_r w[i*R + r] over 16-bit values, R <= 64 (nn.hip)
void sum_repeats(const uint16_t* w, uint16_t* out, int64_t n, int R, hipStream_t st);
void repeat_store(const float* g, float* out, int64_t n_out, int R, bool acc, hipStream_t st);
void gap_bwd(const void* dy, bool dy_f32, uint16_t* dx, int N, int HW, int C, hipStream_t st);
// fused softmax cross-entropy (nn.hip): per-row loss, top-1/top-5 correctness [B][2] and, when
// `grad` is non-null, the logit gradient (softmax - onehot)·gscale (0 for ignored targets)
void xent(const float* logits, const int64_t* target, int B, int C, float gscale,
          int ignore_index, float* loss, float* corr, float* grad, hipStream_t st);
// backward of a fused bias + ReLU epilogue (nn.hip): dym = dy·[y > 0] (y null: no ReLU, dym
// unused) and db (+)= Σ_rows dym; rows [M][C] bf16, C % 8 == 0, C <= 2048; partial holds
// relu_bias_bwd_blocks(M) * C floats
int relu_bias_bwd_blocks(int64_t M, int C);
// several pack_dgrad_kc packs in one launch (conv.hip); prm: 24 ints per job
void pack_kc_multi(const uint16_t* const* w, uint16_t* const* out, const int* prm, int n,
                   hipStream_t st);
// mean cross-entropy [mean, count] of k_xent's rows, and its backward grad · gl / n (nn.hip)
void xent_mean(const float* rows, const int64_t* target, int B, int ignore_index, float* out,
               float* out_n, hipStream_t st);
void xent_scale(const float* grad, const float* gl, const float* n, int64_t total, float* out,
                hipStream_t st);
void relu_bias_bwd(const uint16_t* dy, const uint16_t* y, uint16_t* dym, float* partial,
                   float* db, int64_t M, int C, bool accumulate, hipStream_t st);
void normalize_u8_c4(const uint8_t* in, uint16_t* out, int64_t npix, const float mean[3],
                     const float stdv[3], hipStream_t st);

// CIFAR augmentation (augment.hip): padded NCHW fp32 dataset -> cropped / flipped / cut-out
// NHWC batch (fp32 or bf16); prm is the epoch's [n][5] int32 table (x0, y0, flip, cx, cy)
void cifar_augment(const float* data, const int64_t* idx, const int32_t* prm, void* out, int B,
                   int C, int Hp, int Wp, int crop, int cutout, int64_t offset, bool bf16,
                   hipStream_t st, int Co = 0);

}  // namespace lw
