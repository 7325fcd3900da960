"""Whole-block fused ResNet bottleneck for MI355X training.

The reference runs a bottleneck (``IMAGENET/training/resnet.py:80-118``) as nine separate cuDNN /
ATen ops — conv, BN, ReLU three times, plus the shortcut add — and autograd adds the two gradient
branches of the block input with one more elementwise kernel. On MI355X every one of those ops is
an HBM round trip over a large NHWC activation, and the 1x1 convolutions themselves are
bandwidth-bound (K = 64..512), so the block is organised around the MFMA GEMM of ``csrc/gemm.hip``
and its prologue / epilogue fusions instead:

forward (training)::

    c1 = x·W1ᵀ                       GEMM, epilogue writes BN1 column statistics
    c2 = conv3x3(relu(bn1(c1)))      implicit GEMM (ops/conv.py): BN1-apply+ReLU in the staging
                                     prologue (a1 is never materialised), BN2 stats in the epilogue
    c3 = relu(bn2(c2))·W3ᵀ           GEMM, BN2-apply+ReLU in the prologue, BN3 stats in the epilogue
    [cd = x_s·Wdᵀ                    GEMM + stats (downsample shortcut)]
    out = relu(bn3(c3) + x | bnd(cd)) one pass (the shortcut BN is applied on the fly)

backward::

    bn3 backward (ReLU bitmap)       → dc3   (the shortcut gradient dres = dy·[out>0] is
                                             never written)
    dW3 = dc3ᵀ·relu(bn2(c2))         GEMM, BN2-apply recomputed in the prologue, fp32 written
                                     straight into the gradient arena
    da2 = dc3·W3                     GEMM
    bn2 backward (mask from c2)      → dc2
    dW2 = dc2ᵀ ⋆ relu(bn1(c1))       implicit-GEMM weight gradient, BN1-apply recomputed in the
                                     prologue, split-K, fp32 accumulated into the arena
    da1 = conv3x3ᵀ(dc2)              implicit-GEMM data gradient (stride 2: 4 parity classes)
    bn1 backward (mask from c1)      → dc1
    dW1 = dc1ᵀ·x                     GEMM into the arena
    dx  = dc1·W1 + dy·[out>0]        GEMM; the masked shortcut gradient is added in the epilogue

Compared with the per-layer path this removes, per block, the BN1/BN2/BN3 statistics passes, the
BN1 and BN2 apply passes and their materialised outputs, the shortcut-BN apply pass, the gradient
add of the block input, and the fp32 casts/accumulations of the weight gradients. Every GEMM and
convolution of the block is a hand-written MFMA kernel (no vendor library on this path).

Weight / BN-parameter gradients go **directly into the gradient arena** when the parameter is
owned by a :class:`~..parallel.ddp.CompressedDDP` (which marks it with ``_lw_grad_ready``); the
bucket engine is then notified exactly as a post-accumulate-grad hook would, so compression and
communication still overlap the rest of the backward pass. Without an arena the gradients are
returned through autograd as usual.
"""
from __future__ import annotations

import contextlib
import os
from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

from ._ext import h16, load, set_splitk_defer
from .conv import conv_dgrad, conv_fwd, conv_wgrad, kc_end_step, kc_new_step, kc_pack
from .tuning import MF32, Tuner, with_mf32

CL = torch.channels_last
# materialise relu(bn1(c1)) / relu(bn2(c2)) with one apply pass instead of re-normalising in the
# consumers' staging prologues (see _BottleneckFn.forward)
MAT_A1 = os.environ.get("LWAAAI_MAT_A1", "1") != "0"
MAT_A2 = os.environ.get("LWAAAI_MAT_A2", "1") != "0"
# BN1 / BN2 backward reductions in the epilogues of the data-gradient GEMM / conv producing their
# input gradient (csrc gemm_core.h EPI_BSTATS) instead of a separate pass over dy and x. Off by
# default: it saves the reduce passes (-1.6 ms of BN kernels) but the extra epilogue operands raise
# those GEMMs' registers and serialise their memory phases (+2.4 ms): 9,770 vs 10,297 img/s
# (profiles/r2_bstats_ab.log). LWAAAI_BSTATS=1 / LWAAAI_CROSS_BN3=1 turn the two parts on.
BSTATS = os.environ.get("LWAAAI_BSTATS", "0") == "1"
# The downsample block's BN3 and shortcut-BN backwards share dy and the ReLU bitmap: one dual
# reduce + one dual apply pass (csrc bn.hip k_bn_reduce DUAL / k_bn_bwd_apply_dual) read them once
# for both. LWAAAI_BN_DUAL=0: two separate BN backwards.
BN_DUAL = os.environ.get("LWAAAI_BN_DUAL", "1") != "0"
TILES = with_mf32((1, 2, 3, 4, 5, 6))   # csrc GemmTile ids (0 = heuristic)
STREAM = (11, 12, 13)               # streaming kernel, output panel 64 / 128 / 256
BIG = (21, 22)                      # 256x256 / 256x128 8-wave LDS-DMA kernel (csrc/gemm_big.hip)
# the same tiles as a persistent kernel (csrc/gemm_big.hip k_gemm_bigp: one workgroup per CU, the
# next tile's first K-tiles loaded during this tile's epilogue); LWAAAI_GEMM_PERSIST=0 drops them
PERSIST = (23, 24) if os.environ.get("LWAAAI_GEMM_PERSIST", "1") != "0" else ()


def _rows(t: torch.Tensor) -> torch.Tensor:
    """channels_last NCHW → [N*H*W, C] view (no copy)."""
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


def _nchw(rows: torch.Tensor, n: int, h: int, w: int) -> torch.Tensor:
    return rows.view(n, h, w, rows.shape[1]).permute(0, 3, 1, 2)


# ----------------------------------------------------------------------------- GEMM + tuner
def _splits(tiles: int, K: int) -> int:
    want = max(1, 512 // max(tiles, 1))
    return int(max(1, min(want, K // 256 if K >= 512 else 1)))


def _tile_dims(t: int) -> Tuple[int, int]:
    if MF32 < t <= MF32 + 6:
        t -= MF32
    return {1: (128, 128), 2: (128, 128), 3: (256, 64), 4: (64, 256), 5: (256, 64),
            6: (64, 64), 21: (256, 256), 22: (256, 128), 23: (256, 256), 24: (256, 128)}[t]


class GemmTuner(Tuner):
    """MIOpen-find-style tile selection for the MFMA GEMM: the first time a problem key is seen,
    every tile shape is timed with HIP events on scratch outputs and the fastest is kept for the
    rest of the run. ``LWAAAI_GEMM_TUNE=0`` falls back to the built-in heuristic;
    ``LWAAAI_TUNE_FILE`` pins the choices (``ops/tuning.py``)."""

    def __init__(self):
        super().__init__("gemm", "LWAAAI_GEMM_TUNE")

    def pick(self, key, run, candidates=TILES) -> int:
        return super().pick(key, run, candidates, 0)


TUNER = GemmTuner()


def stream_tiles(M, N, K, a_kc, b_kc, out_bf16, stats, pro, pro_on_a, add, split_k,
                 accumulate) -> tuple:
    """Streaming-kernel candidates for a problem (``csrc/gemm.hip`` k_gemm_stream): large M,
    K in {64, 128, 256}, K-contiguous A, bf16 output; the prologue only with a K-contiguous B."""
    if not (a_kc and out_bf16 and not split_k and not accumulate and M >= 16384 and
            K in (64, 128, 256) and N % 8 == 0 and not (stats and add)):
        return ()
    if pro and (not pro_on_a or not b_kc):
        return ()
    return tuple(t for t in STREAM if not (K == 256 and t == 13))


def gemm(A, lda, a_kc, B, ldb, b_kc, M, N, K, *, out_bf16=True, stats=False, pro=None,
         pro_on_a=True, out=None, addend=None, accumulate=False, ldc=0, split_k=False,
         addend_bits=None, bst=None):
    """One MFMA GEMM launch (plus the split-K reduce when ``split_k``); see ``csrc/gemm.hip``.

    ``bst = (x, mean, scale_shift, bits)``: the output is the gradient reaching a BN+ReLU whose
    input was ``x``; with ``stats=True`` the epilogue also writes that BN backward's per-M-tile
    (Σdy', Σdy'·(x−mean)) rows (mask from ``bits`` or x*scale+shift > 0), which
    ``bn_bwd(..., stats_rows=)`` folds instead of running its reduce pass."""
    lib = load()
    ps, ph = (pro[0], pro[1]) if pro is not None else (None, None)
    bx, bm, bss, bb = bst if bst is not None else (None, None, None, None)

    def splits_for(tile):
        if not split_k:
            return 1
        bm, bn = _tile_dims(tile if tile else 1)
        return _splits(-(-M // bm) * -(-N // bn), K)

    key = (M, N, K, a_kc, b_kc, out_bf16, stats, pro is not None, pro_on_a, split_k,
           addend is not None, bst is not None) + (("sk",) if split_k else ())

    def unpack(c):
        return c if isinstance(c, tuple) else (c, splits_for(c))

    def run(c):
        tile, sp = unpack(c)
        lib.gemm_ex(A, lda, a_kc, B, ldb, b_kc, M, N, K, None, False, sp, out_bf16,
                    tile, ps, ph, pro_on_a, stats, None, addend, False, 0, addend_bits,
                    bx, bm, bss, bb)
    # the big tiles: both operands K-contiguous (forward, transposed-weight dgrad), a K-contiguous
    # A with the weight as stored (dgrad), or both MN-contiguous (weight gradients); no prologue /
    # addend / backward statistics
    big = BIG if (pro is None and addend is None and bst is None and
                  ((a_kc and b_kc and K % 8 == 0) or
                   (a_kc and not b_kc and K % 8 == 0 and N % 8 == 0 and ldb % 8 == 0) or
                   (not a_kc and not b_kc and M % 8 == 0 and N % 8 == 0 and not stats))) else ()
    persist = PERSIST if (pro is None and bst is None and a_kc and b_kc and out_bf16 and
                          not accumulate and not split_k and K % 8 == 0 and K > 64 and
                          N % 8 == 0) else ()
    cands = TILES + big + persist + (() if bst is not None else
                           stream_tiles(M, N, K, a_kc, b_kc, out_bf16, stats, pro is not None,
                                        pro_on_a, addend is not None, split_k, accumulate))
    if split_k:
        # (tile, split-K) pairs: fewer, longer K-slices write fewer fp32 slabs for the fixed-order
        # reduce (the weight gradients are HBM-bound; fewer workgroups can still stream them)
        cands = tuple((t, s) for t in cands
                      for s in sorted({max(1, splits_for(t) >> q) for q in (0, 1, 2, 3)}))
    tile, sp = unpack(TUNER.pick(key, run, cands))
    return lib.gemm_ex(A, lda, a_kc, B, ldb, b_kc, M, N, K, None, False, sp,
                       out_bf16, tile, ps, ph, pro_on_a, stats, out, addend, accumulate, ldc,
                       addend_bits, bx, bm, bss, bb)


LAYOUT_TUNER = Tuner("dgrad-layout", "LWAAAI_GEMM_TUNE")

# 1x1 data-gradient weights in the K-contiguous layout (Wᵀ, gemm_dgrad "kc"): through the per-step
# pack batch of ops/conv.py kc_pack (one k_pack_kc_multi launch for the step's packs).
def new_step() -> None:
    kc_new_step()


def end_step() -> None:
    kc_end_step()


def _kc_weight(W: torch.Tensor, K: int, N: int, kp: int, fresh: bool = False) -> torch.Tensor:
    return kc_pack(W.reshape(K, N, 1, 1), (0, 0, 1, 1), 1, 1, kp,
                   fresh or not W.is_contiguous())


def gemm_dgrad(dy, ldy, W, M, N, K, **kw):
    """Data-gradient GEMM ``dy[M, K] · W[K, N]`` of a 1x1 convolution (W is the forward weight
    [out = K][in = N], N-contiguous as a GEMM B operand). Two layouts are timed on first sight:
    W as stored (the kernel's transposing LDS reads), or Wᵀ copied to [N][K] (a few µs: at most
    2048x512) so that both operands are K-contiguous and the LDS-DMA staging and the big tiles
    apply. ``bst`` (backward statistics) needs the stored layout. (Round 4's opt-in hipBLASLt
    candidate is gone: every kernel of the step is ours.)"""
    def run(layout, fresh=False, **over):
        args = dict(kw, **over)
        if layout == "kc":            # Wᵀ (the tuner times a pack of its own with the GEMM)
            kp = -(-K // 8) * 8
            wt = _kc_weight(W, K, N, kp, fresh)
            return gemm(dy, ldy, True, wt, kp, True, M, N, K, **args)
        return gemm(dy, ldy, True, W, N, False, M, N, K, **args)
    if kw.get("bst") is not None:
        return run("nkc")
    cands = ("nkc", "kc")
    key = (M, N, K, kw.get("addend") is not None, kw.get("out") is not None)
    # timed on a scratch output (``out`` may also be the addend: dx += ... in place)
    layout = LAYOUT_TUNER.pick(key, lambda c: run(c, fresh=True, out=None), cands, "nkc")
    return run(layout)


# ----------------------------------------------------------------------------- cross-block BN3
# The gradient reaching block i's output, dout_i, is the dx written by block i+1's last GEMM. When
# block i+1 has an identity shortcut, that GEMM's epilogue also reduces block i's BN3 backward
# statistics (Σ dout·[out>0], Σ dout·[out>0]·(c3 − mean3)), so block i skips its reduce pass over
# dout and c3. Forward hands block i's (output, c3, mean3, ReLU bitmap) to the next block through
# _FWD_SLOT; backward hands the statistics rows back through _BWD_SLOT, keyed by the gradient
# tensor and checked against block i's own c3, so a mismatch just falls back to the reduce pass.
_FWD_SLOT = [None]
_BWD_SLOT = [None]
CROSS_BN3 = os.environ.get("LWAAAI_CROSS_BN3", "0") == "1"


def _take_prev(x: torch.Tensor):
    prev, _FWD_SLOT[0] = _FWD_SLOT[0], None
    if prev is None or not CROSS_BN3:
        return None
    out_ptr, shape, c3, mean3, bits3 = prev
    if x.data_ptr() != out_ptr or tuple(x.shape) != shape:
        return None
    return c3, mean3, bits3


# ----------------------------------------------------------------------------- grad sink
def _direct(p: torch.Tensor) -> bool:
    """True when ``p.grad`` is an arena view the engine wants written in place."""
    return getattr(p, "_lw_grad_ready", None) is not None and p.grad is not None


def _wgrad_target(p: torch.Tensor, shape) -> Tuple[torch.Tensor, bool]:
    """fp32 [rows, cols] destination for a 1x1-conv weight gradient: the arena view (accumulate)
    or a fresh zero buffer returned through autograd."""
    if _direct(p):
        return p.grad.view(shape), True
    return torch.zeros(shape, dtype=torch.float32, device=p.device), False


def _finish_param(p: torch.Tensor, g: Optional[torch.Tensor], direct: bool):
    """Deliver gradient ``g`` of parameter ``p``: add it into the arena view and notify the
    engine (``g=None``: already accumulated in place), or return it through autograd."""
    if direct:
        if g is not None:
            p.grad.add_(g.view(p.grad.shape))
        p._lw_grad_ready(p)
        return None
    return g.view_as(p) if g is not None else None


def _bn_grad_outs(g: torch.Tensor, b: torch.Tensor):
    """Arena views the BN backward kernel accumulates dgamma/dbeta into (no add kernels), or
    (None, None) when the parameters are not arena-managed."""
    if _direct(g) and _direct(b):
        return g.grad.view(-1), b.grad.view(-1)
    return None, None


def _finish_bn(g: torch.Tensor, b: torch.Tensor, dg, db, outs):
    if outs[0] is not None:          # already accumulated in place by the kernel
        g._lw_grad_ready(g)
        b._lw_grad_ready(b)
        return None, None
    return _finish_param(g, dg, _direct(g)), _finish_param(b, db, _direct(b))


def _finish_wgrad(p: torch.Tensor, dst: torch.Tensor, direct: bool):
    return _finish_param(p, None, True) if direct else dst.view_as(p)


# Weight gradients on a side stream: dW of a layer is independent of the data-gradient chain
# that follows it, so the block's three (four) weight-gradient GEMMs run beside the dgrad GEMMs
# and the latency-bound BN backward kernels instead of between them (fork/join by stream waits;
# inside a HIP-graph capture the fork and join become graph edges). LWAAAI_WGRAD_SIDE=0: inline.
WGRAD_SIDE = os.environ.get("LWAAAI_WGRAD_SIDE", "0") == "1"
_SIDE: Dict[int, torch.cuda.Stream] = {}


class _WgradLane:
    def __init__(self, device: torch.device):
        self.on = WGRAD_SIDE and device.type == "cuda"
        self.main = torch.cuda.current_stream(device) if self.on else None
        if self.on:
            idx = device.index if device.index is not None else torch.cuda.current_device()
            if idx not in _SIDE:
                _SIDE[idx] = torch.cuda.Stream(device=idx)
            self.side = _SIDE[idx]
        self.ready = []
        self.used = False

    def run(self, fn):
        """Launch ``fn`` after everything the main stream has queued so far."""
        if not self.on:
            return fn()
        self.side.wait_stream(self.main)
        with torch.cuda.stream(self.side):
            out = fn()
        self.used = True
        return out

    def finish(self, thunk) -> None:
        """Grad-ready notifications wait for the join (the engine records its bucket events on
        the main stream)."""
        if self.on:
            self.ready.append(thunk)
        else:
            thunk()

    def join(self) -> None:
        if self.on and self.used:
            self.main.wait_stream(self.side)
        for t in self.ready:
            t()
        self.ready = []


# Split-K weight gradients accumulated straight into the gradient arena leave their slab reduce
# to the gradient engine's next flush (csrc/gemm.hip splitk_flush, parallel/engine.py), which
# runs them in one launch before it reads the arena — ResNet-50 spent 54 launches a step on
# these reduces. LWAAAI_SPLITK_DEFER=0: each reduce right after its GEMM.
SPLITK_DEFER = os.environ.get("LWAAAI_SPLITK_DEFER", "1") != "0"


@contextlib.contextmanager
def _deferred_reduce(t: torch.Tensor, direct: bool):
    on = SPLITK_DEFER and direct and t.is_cuda
    if on:
        set_splitk_defer(t, True)
    try:
        yield
    finally:
        if on:
            set_splitk_defer(t, False)


def _wgrad_done(lane: _WgradLane, p: torch.Tensor, dst: torch.Tensor, direct: bool):
    if direct:
        lane.finish(lambda: _finish_param(p, None, True))
        return None
    return dst.view_as(p)


def _bf16_weight(w: torch.Tensor) -> torch.Tensor:
    """bf16 copy of a weight: the view into the arena's per-forward bf16 mirror when it is
    current (``GradArena.refresh_bf16``), else a cast."""
    f = getattr(w, "_lw_bf16_of", None)
    v = f() if f is not None else None
    return v if v is not None else w.detach().to(h16())


def _bn_momentum(bn) -> float:
    if bn.momentum is None:
        return 1.0 / float(bn.num_batches_tracked)
    return float(bn.momentum)


def _bump(bn) -> None:
    if bn.track_running_stats and bn.num_batches_tracked is not None and \
            not getattr(bn, "_shared_counter", False):
        bn.num_batches_tracked.add_(1)


# ----------------------------------------------------------------------------- the block
class _BottleneckFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, g1, b1, w2, g2, b2, w3, g3, b3, wd, gd, bd, mods):
        lib = load()
        bn1, bn2, bn3, conv2, bnd, down_stride = mods
        for bn in (bn1, bn2, bn3) + ((bnd,) if bnd is not None else ()):
            _bump(bn)                 # before the momentum is read (momentum=None: 1/n)
        # the previous block's BN3 state, when x is its output (identity shortcut only)
        ctx.prev = _take_prev(x) if bnd is None else None
        stride = conv2.stride
        N, Cin, H, W = x.shape
        x = x.to(h16()).contiguous(memory_format=CL)
        xr = _rows(x)
        width = w1.shape[0]
        cout = w3.shape[0]
        W1 = _bf16_weight(w1).reshape(width, Cin)
        W2 = _bf16_weight(w2).contiguous(memory_format=CL)
        W3 = _bf16_weight(w3).reshape(cout, width)
        M = xr.shape[0]
        # conv1 (1x1) + BN1 statistics in the epilogue
        c1, st1 = gemm(xr, Cin, True, W1, Cin, True, M, width, Cin, stats=True)
        mean1, inv1, ss1 = lib.bn_stats(c1, st1, g1, b1, bn1.running_mean, bn1.running_var,
                                        _bn_momentum(bn1), bn1.eps)
        # conv2 (3x3, implicit GEMM) on a1 = relu(bn1(c1)), BN2's column statistics in its
        # epilogue. a1 is materialised by one apply pass (MAT_A1): staging-time BN-apply would
        # redo the affine for each of the 9 taps of every element (measured 1.6x slower conv);
        # with MAT_A1=0 the prologue form is used instead.
        pro1 = (ss1[:width], ss1[width:])
        a1 = lib.bn_apply(c1, ss1, None, None, True) if MAT_A1 else None
        c2n, st2 = conv_fwd(_nchw(a1 if MAT_A1 else c1, N, H, W), W2, stride, conv2.padding,
                            pro=None if MAT_A1 else pro1, stats=True)
        N2, _, H2, W2_ = c2n.shape
        c2 = _rows(c2n)
        M2 = c2.shape[0]
        mean2, inv2, ss2 = lib.bn_stats(c2, st2, g2, b2, bn2.running_mean, bn2.running_var,
                                        _bn_momentum(bn2), bn2.eps)
        # conv3 (1x1): BN2-apply+ReLU in the prologue (each A row-panel is re-normalised once
        # per output-column tile) or on a2 materialised by one apply pass (MAT_A2); BN3
        # statistics in the epilogue
        pro2 = (ss2[:width], ss2[width:])
        a2 = lib.bn_apply(c2, ss2, None, None, True) if MAT_A2 else None
        c3, st3 = gemm(a2 if MAT_A2 else c2, width, True, W3, width, True, M2, cout, width,
                       stats=True, pro=None if MAT_A2 else pro2, pro_on_a=True)
        mean3, inv3, ss3 = lib.bn_stats(c3, st3, g3, b3, bn3.running_mean, bn3.running_var,
                                        _bn_momentum(bn3), bn3.eps)
        if bnd is not None:
            s = down_stride
            Wd = _bf16_weight(wd).reshape(cout, Cin)
            if s == 1:
                xsr = xr
                cd, std = gemm(xsr, Cin, True, Wd, Cin, True, M2, cout, Cin, stats=True)
            else:
                # strided 1x1 shortcut as an implicit-GEMM conv gathering every s-th pixel of x
                # (the subsampled input is never materialised)
                xsr = None
                cdn, std = conv_fwd(x, Wd.view(cout, Cin, 1, 1), s, 0, stats=True)
                cd = _rows(cdn)
            meand, invd, ssd = lib.bn_stats(cd, std, gd, bd, bnd.running_mean, bnd.running_var,
                                            _bn_momentum(bnd), bnd.eps)
            bits3 = torch.empty(M2 * cout // 8, dtype=torch.uint8, device=x.device)
            out = lib.bn_apply(c3, ss3, cd, ssd, True, bits3)
            ctx.save_for_backward(x, c1, c2, c3, bits3, W1, W2, W3, g1, g2, g3, mean1, inv1,
                                  ss1, mean2, inv2, ss2, mean3, inv3, a1, a2, xsr, cd, Wd, gd,
                                  meand, invd)
            ctx.down_stride = s
        else:
            bits3 = torch.empty(M2 * cout // 8, dtype=torch.uint8, device=x.device)
            out = lib.bn_apply(c3, ss3, xr, None, True, bits3)
            ctx.save_for_backward(x, c1, c2, c3, bits3, W1, W2, W3, g1, g2, g3, mean1, inv1,
                                  ss1, mean2, inv2, ss2, mean3, inv3, a1, a2)
            ctx.down_stride = 0
        ctx.geom = (N, Cin, H, W, N2, H2, W2_, width, cout, M, M2)
        ctx.conv2 = (list(stride), list(conv2.padding), list(conv2.dilation))
        ctx.params = (w1, g1, b1, w2, g2, b2, w3, g3, b3, wd, gd, bd)
        _FWD_SLOT[0] = (out.data_ptr(), (N2, cout, H2, W2_), c3, mean3, bits3)
        return _nchw(out, N2, H2, W2_)

    @staticmethod
    def backward(ctx, dout):
        lib = load()
        saved = ctx.saved_tensors
        x, c1, c2, c3, bits3, W1, W2, W3, g1, g2, g3, mean1, inv1, ss1, mean2, inv2, ss2, \
            mean3, inv3, a1, a2 = saved[:21]
        N, Cin, H, W, N2, H2, W2_, width, cout, M, M2 = ctx.geom
        w1, g1p, b1p, w2, g2p, b2p, w3, g3p, b3p, wd, gdp, bdp = ctx.params
        has_down = ctx.down_stride > 0
        dr = _rows(dout.to(h16()).contiguous(memory_format=CL))
        # BN3 (+ shortcut) backward, ReLU mask from the forward's 1-bit bitmap
        o3 = _bn_grad_outs(g3p, b3p)
        # (the shortcut gradient dy·[out>0] is never materialised: its consumers read dy and
        # the bitmap — the dx GEMM as a masked addend, the shortcut BN through its ReLU mode)
        rows3 = None
        slot, _BWD_SLOT[0] = _BWD_SLOT[0], None
        if slot is not None and slot[0] == dr.data_ptr() and slot[2] == c3.data_ptr():
            rows3 = slot[1]             # reduced by the next block's dx GEMM epilogue
        grads = {}
        dual = None
        if has_down and BN_DUAL and rows3 is None:
            cd, gd, meand, invd = saved[22], saved[24], saved[25], saved[26]
            od = _bn_grad_outs(gdp, bdp)
            dc3, dcd, dg3, db3, dgd, dbd = lib.bn_bwd_dual(dr, c3, cd, bits3, g3, mean3, inv3, gd,
                                                           meand, invd, o3[0], o3[1], od[0],
                                                           od[1])
            dual = (dcd, dgd, dbd, od)
        else:
            dc3, dg3, db3, _ = lib.bn_bwd(dr, c3, None, g3, mean3, inv3, None, True, True, False,
                                          bits3, o3[0], o3[1], rows3)
        grads["g3"], grads["b3"] = _finish_bn(g3p, b3p, dg3, db3, o3)
        # conv3: weight gradient on a2 (or with BN2-apply recomputed in the B prologue), fp32
        # accumulated into the arena
        lane = _WgradLane(dc3.device)
        dst3, d3 = _wgrad_target(w3, (cout, width))
        with _deferred_reduce(dc3, d3):
            lane.run(lambda: gemm(dc3, cout, False, c2 if a2 is None else a2, width, False, cout,
                                  width, M2, out_bf16=False,
                                  pro=(ss2[:width], ss2[width:]) if a2 is None else None,
                                  pro_on_a=False, out=dst3, accumulate=True, split_k=True))
        grads["w3"] = _wgrad_done(lane, w3, dst3, d3)
        # da2 = dc3·W3, its epilogue doing BN2's backward reduction (mask from c2 via ss2)
        da2, rows2 = gemm_dgrad(dc3, cout, W3, M2, width, cout, stats=BSTATS,
                                bst=(c2, mean2, ss2, None) if BSTATS else None)
        o2 = _bn_grad_outs(g2p, b2p)
        dc2, dg2, db2, _ = lib.bn_bwd(da2, c2, None, g2, mean2, inv2, ss2, True, True, False,
                                      None, o2[0], o2[1], rows2 if BSTATS else None)
        grads["g2"], grads["b2"] = _finish_bn(g2p, b2p, dg2, db2, o2)
        # conv2 (3x3) backward on the implicit GEMM: the weight gradient reads a1 (or
        # recomputes relu(bn1(c1)) in its staging prologue) and accumulates fp32 straight into
        # the arena
        stride, padding, dilation = ctx.conv2
        dc2n = _nchw(dc2, N2, H2, W2_)
        c1n = _nchw(c1 if a1 is None else a1, N, H, W)
        pro1 = (ss1[:width], ss1[width:]) if a1 is None else None
        if _direct(w2) and w2.grad.is_contiguous(memory_format=CL):
            with _deferred_reduce(dc2n, True):
                lane.run(lambda: conv_wgrad(dc2n, c1n, tuple(w2.shape), stride, padding, pro=pro1,
                                            out=w2.grad))
            lane.finish(lambda: _finish_param(w2, None, True))
            grads["w2"] = None
        else:
            dW2 = lane.run(lambda: conv_wgrad(dc2n, c1n, tuple(w2.shape), stride, padding,
                                              pro=pro1).contiguous(memory_format=CL))
            if _direct(w2):
                lane.finish(lambda: _finish_param(w2, dW2, True))
                grads["w2"] = None
            else:
                grads["w2"] = dW2.view_as(w2)
        # da1 = conv3x3ᵀ(dc2), its epilogue doing BN1's backward reduction
        if BSTATS:
            da1n, rows1 = conv_dgrad(dc2n, W2, (H, W), stride, padding, bst=(c1, mean1, ss1, None))
        else:
            da1n, rows1 = conv_dgrad(dc2n, W2, (H, W), stride, padding), None
        da1 = _rows(da1n)
        o1 = _bn_grad_outs(g1p, b1p)
        dc1, dg1, db1, _ = lib.bn_bwd(da1, c1, None, g1, mean1, inv1, ss1, True, True, False,
                                      None, o1[0], o1[1], rows1)
        grads["g1"], grads["b1"] = _finish_bn(g1p, b1p, dg1, db1, o1)
        xr = _rows(x)
        dst1, d1 = _wgrad_target(w1, (width, Cin))
        with _deferred_reduce(dc1, d1):
            lane.run(lambda: gemm(dc1, width, False, xr, Cin, False, width, Cin, M,
                                  out_bf16=False, out=dst1, accumulate=True, split_k=True))
        grads["w1"] = _wgrad_done(lane, w1, dst1, d1)
        if has_down:
            xsr, cd, Wd, gd, meand, invd = saved[21:]
            s = ctx.down_stride
            if dual is not None:
                dcd, dgd, dbd, od = dual
            else:
                od = _bn_grad_outs(gdp, bdp)
                dcd, dgd, dbd, _ = lib.bn_bwd(dr, cd, None, gd, meand, invd, None, True, True,
                                              False, bits3, od[0], od[1])
            grads["gd"], grads["bd"] = _finish_bn(gdp, bdp, dgd, dbd, od)
            dstd, dd = _wgrad_target(wd, (cout, Cin))
            with _deferred_reduce(dcd, dd):
                if s == 1:
                    lane.run(lambda: gemm(dcd, cout, False, xsr, Cin, False, cout, Cin, M2,
                                          out_bf16=False, out=dstd, accumulate=True,
                                          split_k=True))
                else:                 # strided pixel gather of x in the weight-gradient conv
                    lane.run(lambda: conv_wgrad(_nchw(dcd, N2, H2, W2_), x, (cout, Cin, 1, 1), s,
                                                0, out=dstd.view(cout, Cin, 1, 1)))
            grads["wd"] = _wgrad_done(lane, wd, dstd, dd)
            dx, _ = gemm_dgrad(dc1, width, W1, M, Cin, width)
            if s == 1:
                gemm_dgrad(dcd, cout, Wd, M2, Cin, cout, out=dx, addend=dx)
            else:
                # the shortcut's data gradient lands on every s-th pixel of dx: a 1-class
                # strided data-gradient conv adding into dx in place (no scatter pass)
                conv_dgrad(_nchw(dcd, N2, H2, W2_), Wd.view(cout, Cin, 1, 1), (H, W), s, 0,
                           out=dx, addend=dx)
        else:
            prev = ctx.prev           # the previous block's (c3, mean3, bits3): reduce its BN3
            dx, rows_prev = gemm_dgrad(dc1, width, W1, M, Cin, width, addend=dr,
                                       addend_bits=bits3, stats=prev is not None,
                                       bst=(prev[0], prev[1], None, prev[2]) if prev is not None
                                       else None)
            if prev is not None:
                _BWD_SLOT[0] = (dx.data_ptr(), rows_prev, prev[0].data_ptr())
        ctx.prev = None
        lane.join()                   # the weight gradients are done before anything reads them
        dxn = _nchw(dx, N, H, W)
        return (dxn, grads["w1"], grads["g1"], grads["b1"], grads["w2"], grads["g2"], grads["b2"],
                grads["w3"], grads["g3"], grads["b3"], grads.get("wd"), grads.get("gd"),
                grads.get("bd"), None)


def block_supported(m, x: torch.Tensor) -> bool:
    """The fused path needs a CUDA bf16-able channels_last input, BN with affine params and
    running stats, 8-aligned channel counts and a plain 1x1 / 3x3 / 1x1 bottleneck."""
    if not (x.is_cuda and x.dim() == 4 and m.training):
        return False
    bns = [m.bn1, m.bn2, m.bn3] + ([m.downsample[1]] if m.downsample is not None else [])
    if any(not (b.affine and b.track_running_stats) for b in bns):
        return False
    if any(c.groups != 1 for c in (m.conv1, m.conv2, m.conv3)):
        return False
    chans = [x.shape[1], m.conv1.out_channels, m.conv3.out_channels]
    return all(c % 8 == 0 for c in chans)


def bottleneck_forward(m, x: torch.Tensor) -> torch.Tensor:
    """Training forward of a ``models.resnet.Bottleneck`` through :class:`_BottleneckFn`."""
    down = m.downsample
    if down is not None:
        wd, bnd = down[0].weight, down[1]
        gd, bd, ds = bnd.weight, bnd.bias, down[0].stride[0]
    else:
        wd = gd = bd = bnd = None
        ds = 0
    mods = (m.bn1, m.bn2, m.bn3, m.conv2, bnd, ds)
    with torch.autocast("cuda", enabled=False):
        return _BottleneckFn.apply(x, m.conv1.weight, m.bn1.weight, m.bn1.bias, m.conv2.weight,
                                   m.bn2.weight, m.bn2.bias, m.conv3.weight, m.bn3.weight,
                                   m.bn3.bias, wd, gd, bd, mods)
