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
# Design decisions measured in earlier rounds and fixed in round 6 (their switches removed):
# * relu(bn1(c1)) is materialised by one apply pass, not re-normalised in the 3x3 conv's staging
#   (it would redo the affine for each of its 9 taps: 1.6x slower); relu(bn2(c2)) likewise at
#   stages 3-4, while at stages 1-2 conv3 applies BN2 in its GEMM prologue and the fused BN3
#   backward re-forms a2 from c2, so a2 is never written;
# * the BN backward reductions run as their own pass: folding them into the epilogue of the GEMM
#   producing dy saved 1.6 ms of BN kernels but cost 2.4 ms of GEMM (profiles/r2_bstats_ab.log;
#   -3.3 % each part, profiles/r3s2/bstats_cross_ab.txt);
# * the downsample block's BN3 and shortcut-BN backwards share dy and the ReLU bitmap: one dual
#   reduce + one dual apply pass (csrc bn.hip k_bn_reduce DUAL / k_bn_bwd_apply_dual);
# * weight gradients run inline (a side stream measured no gain: the step is throughput-bound).
# * the BN3 backward of a 256- or 512-channel block (ResNet-50 stages 1-2) runs its apply inside
#   one kernel with both GEMMs that read dc3 (csrc/bnfuse.hip): dy, c3 and the bitmap are read
#   once instead of dc3 being written and read twice; 604.2 -> 417.1 us a stage-1 block, 327.4 ->
#   272.2 us a stage-2 block, bench 11,738 -> 12,173 img/s on one box (profiles/r6/fused_bn3/);
#   likewise BN1 of a block without downsample with dW1 = dc1ᵀ·x and dx = dc1·W1 + dy·bit3.
#   LWAAAI_FUSE_BNBWD=0: the three passes.
FUSE_BNBWD = os.environ.get("LWAAAI_FUSE_BNBWD", "1") != "0"
TILES = with_mf32((1, 2, 3, 4, 5, 6))   # csrc GemmTile ids (0 = heuristic)
STREAM = (11, 12, 13)               # streaming kernel, output panel 64 / 128 / 256
BIG = (21, 22)                      # 256x256 / 256x128 8-wave LDS-DMA kernel (csrc/gemm_big.hip)
# the same tiles as a persistent kernel (csrc/gemm_big.hip k_gemm_bigp: one workgroup per CU, the
# next tile's first K-tiles loaded during this tile's epilogue)
PERSIST = (23, 24)


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
         addend_bits=None):
    """One MFMA GEMM launch (plus the split-K reduce when ``split_k``); see ``csrc/gemm.hip``."""
    lib = load()
    ps, ph = (pro[0], pro[1]) if pro is not None else (None, None)

    def splits_for(tile):
        if not split_k:
            return 1
        bm, bn = _tile_dims(tile if tile else 1)
        return _splits(-(-M // bm) * -(-N // bn), K)

    key = (M, N, K, a_kc, b_kc, out_bf16, stats, pro is not None, pro_on_a, split_k,
           addend is not None, False) + (("sk",) if split_k else ())

    def unpack(c):
        return c if isinstance(c, tuple) else (c, splits_for(c))

    def run(c):
        tile, sp = unpack(c)
        lib.gemm_ex(A, lda, a_kc, B, ldb, b_kc, M, N, K, None, False, sp, out_bf16,
                    tile, ps, ph, pro_on_a, stats, None, addend, False, 0, addend_bits)
    # the big tiles: both operands K-contiguous (forward, transposed-weight dgrad), a K-contiguous
    # A with the weight as stored (dgrad), or both MN-contiguous (weight gradients); no prologue /
    # addend
    big = BIG if (pro is None and addend is None and
                  ((a_kc and b_kc and K % 8 == 0) or
                   (a_kc and not b_kc and K % 8 == 0 and N % 8 == 0 and ldb % 8 == 0) or
                   (not a_kc and not b_kc and M % 8 == 0 and N % 8 == 0 and not stats))) else ()
    persist = PERSIST if (pro is None and a_kc and b_kc and out_bf16 and
                          not accumulate and not split_k and K % 8 == 0 and K > 64 and
                          N % 8 == 0) else ()
    cands = TILES + big + persist + stream_tiles(M, N, K, a_kc, b_kc, out_bf16, stats,
                                                 pro is not None, pro_on_a, addend is not None,
                                                 split_k, accumulate)
    if split_k:
        # (tile, split-K) pairs: fewer, longer K-slices write fewer fp32 slabs for the fixed-order
        # reduce (the weight gradients are HBM-bound; fewer workgroups can still stream them)
        cands = tuple((t, s) for t in cands
                      for s in sorted({max(1, splits_for(t) >> q) for q in (0, 1, 2, 3)}))
    tile, sp = unpack(TUNER.pick(key, run, cands))
    return lib.gemm_ex(A, lda, a_kc, B, ldb, b_kc, M, N, K, None, False, sp,
                       out_bf16, tile, ps, ph, pro_on_a, stats, out, addend, accumulate, ldc,
                       addend_bits)


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
    apply. (Round 4's opt-in hipBLASLt candidate is gone: every kernel of the step is ours.)"""
    def run(layout, fresh=False, **over):
        args = dict(kw, **over)
        if layout == "kc":            # Wᵀ (the tuner times a pack of its own with the GEMM)
            kp = -(-K // 8) * 8
            wt = _kc_weight(W, K, N, kp, fresh)
            return gemm(dy, ldy, True, wt, kp, True, M, N, K, **args)
        return gemm(dy, ldy, True, W, N, False, M, N, K, **args)
    cands = ("nkc", "kc")
    key = (M, N, K, kw.get("addend") is not None, kw.get("out") is not None)
    # timed on a scratch output (``out`` may also be the addend: dx += ... in place)
    layout = LAYOUT_TUNER.pick(key, lambda c: run(c, fresh=True, out=None), cands, "nkc")
    return run(layout)


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


# Split-K weight gradients accumulated straight into the gradient arena leave their slab reduce
# to the gradient engine's next flush (csrc/gemm.hip splitk_flush, parallel/engine.py), which
# runs them in one launch before it reads the arena — ResNet-50 spent 54 launches a step on
# these reduces (profiles/r5/splitk_defer_ab.jsonl).
@contextlib.contextmanager
def _deferred_reduce(t: torch.Tensor, direct: bool):
    on = direct and t.is_cuda
    if on:
        set_splitk_defer(t, True)
    try:
        yield
    finally:
        if on:
            set_splitk_defer(t, False)


def _wgrad_done(p: torch.Tensor, dst: torch.Tensor, direct: bool):
    if direct:
        _finish_param(p, None, True)
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
        # conv2 (3x3, implicit GEMM) on a1 = relu(bn1(c1)), materialised by one apply pass, BN2's
        # column statistics in its epilogue
        a1 = lib.bn_apply(c1, ss1, None, None, True)
        c2n, st2 = conv_fwd(_nchw(a1, N, H, W), W2, stride, conv2.padding, stats=True)
        N2, _, H2, W2_ = c2n.shape
        c2 = _rows(c2n)
        M2 = c2.shape[0]
        mean2, inv2, ss2 = lib.bn_stats(c2, st2, g2, b2, bn2.running_mean, bn2.running_var,
                                        _bn_momentum(bn2), bn2.eps)
        # conv3 (1x1) on a2 = relu(bn2(c2)), BN3 statistics in the epilogue. Where BN3's backward
        # runs fused (stages 1-2) a2 is never materialised: the GEMM applies BN2 + ReLU as it
        # stages c2 (the apply kernel's expression, bit for bit) and the fused backward re-forms
        # a2 from c2 the same way (12,387-12,396 -> 12,456-12,469 img/s alternating on one box,
        # profiles/r6/a2free/)
        fuse3 = FUSE_BNBWD and (cout, width) in ((256, 64), (512, 128)) and c2.dtype == h16()
        if fuse3:
            a2 = c2
            c3, st3 = gemm(c2, width, True, W3, width, True, M2, cout, width, stats=True,
                           pro=(ss2[:width], ss2[width:]))
        else:
            a2 = lib.bn_apply(c2, ss2, None, None, True)
            c3, st3 = gemm(a2, width, True, W3, width, True, M2, cout, width, stats=True)
        ctx.fuse3 = fuse3
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
        grads = {}
        dual = None
        st2 = None
        fused = ctx.fuse3             # (decided by the forward: a2 is c2 then)
        if fused:
            # BN3's apply fused into both consumers of dc3 (csrc/bnfuse.hip): da2 = dc3·W3 and
            # dW3 = dc3ᵀ·a2 from one pass over dy, c3 and the bitmap; dc3 is never written (a
            # downsample block's shortcut-BN gradient dcd comes out of the same pass)
            dst3, d3 = _wgrad_target(w3, (cout, width))
            w3t = _kc_weight(W3, cout, width, cout).view(width, cout)
            down = ()
            if has_down:
                cd, gd, meand, invd = saved[22], saved[24], saved[25], saved[26]
                od = _bn_grad_outs(gdp, bdp)
                down = (cd, gd, meand, invd, od[0], od[1])
            if not has_down:
                down = (None,) * 6
            # stage 1: BN2's backward sums come out of the same kernel, from the da2 tiles it
            # writes: the bandwidth-bound kernel reads c2 (+29 us a block in the step) and BN2's
            # reduce pass over da2 and c2 (45 us) is gone: 20.769 -> 20.704 ms of kernels a
            # step. At stage 2 they cost the kernel more than the pass they replace (292.9 vs
            # 271.2 us in isolation). profiles/r6/bn2_sums/
            s2 = (c2, ss2, mean2) if cout == 256 else (None, ss2, None)
            with _deferred_reduce(dr, d3):
                da2, _, dg3, db3, dcd, dgd, dbd, st2 = lib.bn3_bwd_fused(
                    dr, c3, bits3, g3, mean3, inv3, w3t, c2, dst3, o3[0], o3[1], *down, *s2,
                    True)
                if s2[0] is None:
                    st2 = None
            if has_down:
                dual = (dcd, dgd, dbd, od)
            grads["g3"], grads["b3"] = _finish_bn(g3p, b3p, dg3, db3, o3)
            grads["w3"] = _wgrad_done(w3, dst3, d3)
        elif has_down:
            cd, gd, meand, invd = saved[22], saved[24], saved[25], saved[26]
            od = _bn_grad_outs(gdp, bdp)
            dc3, dcd, dg3, db3, dgd, dbd = lib.bn_bwd_dual(dr, c3, cd, bits3, g3, mean3, inv3, gd,
                                                           meand, invd, o3[0], o3[1], od[0],
                                                           od[1])
            dual = (dcd, dgd, dbd, od)
        else:
            dc3, dg3, db3, _ = lib.bn_bwd(dr, c3, None, g3, mean3, inv3, None, True, True, False,
                                          bits3, o3[0], o3[1])
        if "w3" not in grads:
            grads["g3"], grads["b3"] = _finish_bn(g3p, b3p, dg3, db3, o3)
            # conv3: weight gradient on a2, fp32 accumulated into the arena
            dst3, d3 = _wgrad_target(w3, (cout, width))
            with _deferred_reduce(dc3, d3):
                gemm(dc3, cout, False, a2, width, False, cout, width, M2, out_bf16=False,
                     out=dst3, accumulate=True, split_k=True)
            grads["w3"] = _wgrad_done(w3, dst3, d3)
            # da2 = dc3·W3
            da2, _ = gemm_dgrad(dc3, cout, W3, M2, width, cout)
        o2 = _bn_grad_outs(g2p, b2p)
        dc2, dg2, db2, _ = lib.bn_bwd(da2, c2, None, g2, mean2, inv2, ss2, True, True, False,
                                      None, o2[0], o2[1], st2)
        grads["g2"], grads["b2"] = _finish_bn(g2p, b2p, dg2, db2, o2)
        # conv2 (3x3) backward on the implicit GEMM: the weight gradient reads a1 and accumulates
        # fp32 straight into the arena
        stride, padding, dilation = ctx.conv2
        dc2n = _nchw(dc2, N2, H2, W2_)
        a1n = _nchw(a1, N, H, W)
        if _direct(w2) and w2.grad.is_contiguous(memory_format=CL):
            with _deferred_reduce(dc2n, True):
                conv_wgrad(dc2n, a1n, tuple(w2.shape), stride, padding, out=w2.grad)
            _finish_param(w2, None, True)
            grads["w2"] = None
        else:
            dW2 = conv_wgrad(dc2n, a1n, tuple(w2.shape), stride, padding).contiguous(
                memory_format=CL)
            if _direct(w2):
                _finish_param(w2, dW2, True)
                grads["w2"] = None
            else:
                grads["w2"] = dW2.view_as(w2)
        # da1 = conv3x3ᵀ(dc2)
        da1 = _rows(conv_dgrad(dc2n, W2, (H, W), stride, padding))
        o1 = _bn_grad_outs(g1p, b1p)
        if (FUSE_BNBWD and not has_down and (width, Cin) in ((64, 256), (128, 512)) and
                dr.dtype == h16()):
            # BN1's apply fused into both consumers of dc1 (csrc/bnfuse.hip): dx = dc1·W1 +
            # dy·bit3 and dW1 = dc1ᵀ·x from one pass; dc1 is never written
            dst1, d1 = _wgrad_target(w1, (width, Cin))
            with _deferred_reduce(da1, d1):
                dx, _, dg1, db1 = lib.bn1_bwd_fused(
                    da1, c1, ss1, g1, mean1, inv1,
                    _kc_weight(W1, width, Cin, width).view(Cin, width), _rows(x), dr, bits3,
                    dst1, o1[0], o1[1])
            grads["g1"], grads["b1"] = _finish_bn(g1p, b1p, dg1, db1, o1)
            grads["w1"] = _wgrad_done(w1, dst1, d1)
            return (_nchw(dx, N, H, W), grads["w1"], grads["g1"], grads["b1"], grads["w2"],
                    grads["g2"], grads["b2"], grads["w3"], grads["g3"], grads["b3"], None, None,
                    None, None)
        dc1, dg1, db1, _ = lib.bn_bwd(da1, c1, None, g1, mean1, inv1, ss1, True, True, False,
                                      None, o1[0], o1[1])
        grads["g1"], grads["b1"] = _finish_bn(g1p, b1p, dg1, db1, o1)
        xr = _rows(x)
        dst1, d1 = _wgrad_target(w1, (width, Cin))
        with _deferred_reduce(dc1, d1):
            gemm(dc1, width, False, xr, Cin, False, width, Cin, M, out_bf16=False, out=dst1,
                 accumulate=True, split_k=True)
        grads["w1"] = _wgrad_done(w1, dst1, d1)
        if has_down:
            xsr, cd, Wd, gd, meand, invd = saved[21:]
            s = ctx.down_stride
            dcd, dgd, dbd, od = dual
            grads["gd"], grads["bd"] = _finish_bn(gdp, bdp, dgd, dbd, od)
            dstd, dd = _wgrad_target(wd, (cout, Cin))
            with _deferred_reduce(dcd, dd):
                if s == 1:
                    gemm(dcd, cout, False, xsr, Cin, False, cout, Cin, M2, out_bf16=False,
                         out=dstd, accumulate=True, split_k=True)
                else:                 # strided pixel gather of x in the weight-gradient conv
                    conv_wgrad(_nchw(dcd, N2, H2, W2_), x, (cout, Cin, 1, 1), s, 0,
                               out=dstd.view(cout, Cin, 1, 1))
            grads["wd"] = _wgrad_done(wd, dstd, dd)
            dx, _ = gemm_dgrad(dc1, width, W1, M, Cin, width)
            if s == 1:
                gemm_dgrad(dcd, cout, Wd, M2, Cin, cout, out=dx, addend=dx)
            else:
                # the shortcut's data gradient lands on every s-th pixel of dx: a 1-class
                # strided data-gradient conv adding into dx in place (no scatter pass)
                conv_dgrad(_nchw(dcd, N2, H2, W2_), Wd.view(cout, Cin, 1, 1), (H, W), s, 0,
                           out=dx, addend=dx)
        else:
            # dx = dc1·W1 + dy·[out>0]: the masked shortcut gradient added in the epilogue
            dx, _ = gemm_dgrad(dc1, width, W1, M, Cin, width, addend=dr, addend_bits=bits3)
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
