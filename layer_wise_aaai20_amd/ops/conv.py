"""Hand-written MFMA implicit-GEMM convolutions (``csrc/conv.hip``) and the layer built on them.

Every convolution of the reference models — the ResNet-50 3x3 bottleneck convs and 7x7 stem
(``IMAGENET/training/resnet.py:18-21,63-64,100``), the ResNet-9 / AlexNet / VGG-16 CIFAR convs
(``CIFAR10/dawn.py:23-33``, ``CIFAR10/alexnet.py:15-25``, ``CIFAR10/vgg16.py:76``) — runs its
forward, data gradient and weight gradient here, on the same MFMA GEMM core as the 1x1 convs and
Linear layers, with NHWC bf16 activations and fp32 accumulation:

  * forward: ``y = im2col(x)·Wᵀ`` with the window gathered while staging (no im2col buffer); an
    optional BatchNorm-apply+ReLU of the input in the staging prologue and the next BN's column
    statistics in the epilogue;
  * data gradient: the transposed conv as a gather over dY with the taps walked backwards; a
    stride-2 conv runs as its 4 output-parity classes, each a dense stride-1 GEMM over the taps
    that reach it;
  * weight gradient: split-K over the output pixels with fp32 written (or accumulated) straight
    into the gradient arena view of a channels_last weight ([Co][R][S][C] = the GEMM output).

A 3-channel input (the image) runs as a 4-channel one whose chunks are two adjacent taps.
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch
import torch.nn.functional as F
from torch import nn

from ._ext import h16, load
from .tuning import MF32, Tuner, with_mf32

CL = torch.channels_last
CV_A, CV_A4, CV_B, CV_B4 = 1, 2, 3, 4
# forward / dgrad and weight-gradient tiles (csrc GemmTile ids), each with its 32x32x16-MFMA twin
# (id + 40, ops/block.py with_mf32)
ROW_TILES = with_mf32((1, 2, 3, 5, 6))
COL_TILES = with_mf32((1, 2, 4, 6))
# 256x256 / 256x128 8-wave LDS-DMA tiles (csrc/gemm_big.hip, row gather): one stride-1 class,
# C % 64 == 0 (a K-tile inside one tap), K-contiguous weight, no prologue / addend / statistics
# of the backward
BIG_TILES = (21, 22)
# the direct 7x7/2 stem convolution from an LDS patch (csrc/conv.hip k_stem_conv7), a tuner
# candidate of the ResNet stem's forward (337 vs 392 us at bs 256, profiles/r3s2/). (A direct
# 3x3/1 64-channel kernel from an LDS patch measured 130 / 151 us against 127 / 117 us for the
# implicit GEMM, profiles/r3s2/direct_probe.txt, and was removed in round 6.)
STEM_DIRECT = 31
# the tap-reuse 3x3/1 convolution (csrc/conv3tap.hip k_conv3_tap): the input patch of a
# 224-pixel tile is staged once per 32-channel chunk and read by all 9 taps (the implicit GEMM
# gathers it 9 times), forward and — flipped, transposed weight — data gradient. C % 32 == 0,
# Co == 64 or Co % 128 == 0, image width dividing 224.
CONV3_TAP = 33
# (A weight-resident persistent form for C = Co = 64 — the whole 72 KB weight in LDS, one
# workgroup per CU, no barrier inside a tile — measured 130.6 / 121.3 us against this kernel's
# 122.2 / 111.5 at 56x56, batch 256 (profiles/r6/conv3_res_ab.txt), and was removed in round 6.)


def _conv3_tap_fits(c, co, R, S, sh, sw, ph, pw, H, W) -> bool:
    if not ((R, S) == (3, 3) and (sh, sw) == (1, 1) and (ph, pw) == (1, 1)):
        return False
    if c % 32 or c < 32 or not (co == 64 or co % 128 == 0) or W < 4 or 224 % W:
        return False
    rows = 224 // W
    return ((rows + 2) * W + 2) * 64 <= 24 * 1024


# K-contiguous data-gradient weight packs (csrc/conv.hip k_pack_dgrad_kc: 1x1 transposes Wᵀ, the
# strided / 3x3 class slabs, the flipped 3x3 window) batched per step: at a step's first request
# every pack asked for in the last step is made in one launch (k_pack_kc_multi; ResNet-50 ran ~15
# pack launches a step), a pack not seen before runs alone and joins. The registry holds the weight
# tensors (the bf16 mirror's views, refreshed in place every step, or bf16 parameters updated in
# place), so a key's data pointer cannot be reused by another tensor while listed; entries not
# asked for in a step are dropped. Only between the gradient engine's begin_step (kc_new_step)
# and its finish (kc_end_step): a backward outside an engine step packs per request.
_KC = {"gen": -1, "armed": False, "reg": {}, "cache": {}, "used": set()}
_STEP_GEN = [0]


def kc_new_step() -> None:
    _STEP_GEN[0] += 1
    _KC["armed"] = True


def kc_end_step() -> None:
    _KC["armed"] = False


def _pack1(lib, wb, cls, sh, sw, kmax):
    if kmax == 0:
        return lib.pack_dgrad_nkc(wb, list(cls), sh, sw)
    return lib.pack_dgrad_kc(wb, list(cls), sh, sw, kmax)


def kc_pack(wb: torch.Tensor, cls, sh: int, sw: int, kmax: int, fresh: bool = False):
    """``pack_dgrad_kc(wb, cls, sh, sw, kmax)`` — or ``pack_dgrad_nkc(wb, cls, sh, sw)`` for
    ``kmax == 0`` — through the per-step batch (``fresh``: a pack of its own, e.g. timed by the
    tuner with its GEMM)."""
    lib = load()
    if fresh or not _KC["armed"] or not wb.is_cuda:
        return _pack1(lib, wb, cls, sh, sw, kmax)
    key = (wb.data_ptr(), tuple(wb.shape), tuple(cls), sh, sw, kmax)
    if _KC["gen"] != _STEP_GEN[0]:
        _KC["gen"] = _STEP_GEN[0]
        # (a model of the other precision's build, or on another device, may have filled it)
        _KC["reg"] = {k: w for k, w in _KC["reg"].items()
                      if k in _KC["used"] and w.dtype == wb.dtype and w.device == wb.device}
        _KC["used"] = set()
        _KC["cache"] = {}
        reg = list(_KC["reg"].items())
        if reg:
            outs, prm = [], []
            for k, w in reg:
                c4 = list(k[2]) + [0] * (16 - len(k[2]))
                nc = len(k[2]) // 4
                n = (nc * w.shape[1] * k[5] if k[5] else
                     sum(c4[4 * i + 2] * c4[4 * i + 3] for i in range(nc)) * w.shape[0] * w.shape[1])
                outs.append(torch.empty(n, dtype=w.dtype, device=w.device))
                prm += [k[3], k[4], k[5], nc] + c4[0::4] + c4[1::4] + c4[2::4] + c4[3::4]
            lib.pack_kc_multi([w for _, w in reg], outs, prm)
            _KC["cache"] = {k: o for (k, _), o in zip(reg, outs)}
    _KC["used"].add(key)
    hit = _KC["cache"].get(key)
    if hit is not None:
        return hit
    out = _pack1(lib, wb, cls, sh, sw, kmax)
    _KC["reg"][key] = wb
    _KC["cache"][key] = out
    return out


def tap_dgrad_weight(w: torch.Tensor, fresh: bool = True) -> torch.Tensor:
    """The data gradient of a 3x3/1/1 conv as a forward conv of dy: W'[ci][r][s][co] =
    w[co][ci][2-r][2-s], K-contiguous [C][9 Co]."""
    co, c, R, S = w.shape
    wb = w.to(h16())
    if (wb.is_cuda and (R, S) == (3, 3) and co % 8 == 0 and
            wb.is_contiguous(memory_format=CL)):
        # one pack kernel walking the window backwards (was flip + two copies, ~15 µs a call)
        return kc_pack(wb, [2, 2, 3, 3], -1, -1, 9 * co, fresh or wb is not w).view(c, 9 * co)
    return wb.flip(2, 3).permute(1, 2, 3, 0).reshape(c, -1).contiguous()


_TILE_DIMS = {1: (128, 128, 32), 2: (128, 128, 64), 3: (256, 64, 32), 4: (64, 256, 32),
              5: (256, 64, 64), 6: (64, 64, 64), 21: (256, 256, 64), 22: (256, 128, 64)}
_TILE_DIMS.update({MF32 + t: _TILE_DIMS[t] for t in range(1, 7)})


def _pair(v) -> Tuple[int, int]:
    return (v, v) if isinstance(v, int) else (int(v[0]), int(v[1]))


def out_size(h: int, k: int, s: int, p: int) -> int:
    return (h + 2 * p - k) // s + 1


def supported(cin: int, cout: int, groups: int = 1, dilation=(1, 1)) -> bool:
    return groups == 1 and tuple(_pair(dilation)) == (1, 1) and cout % 8 == 0 and \
        (cin % 8 == 0 or cin in (3, 4))


# ----------------------------------------------------------------------------- tile tuner
class ConvTuner(Tuner):
    """First sight of a problem key: time every candidate (tile, or (tile, splits)) with HIP
    events on scratch outputs and keep the fastest — MIOpen-find-style, but over our own
    kernels only. ``LWAAAI_GEMM_TUNE=0`` keeps the heuristic choice; ``LWAAAI_TUNE_FILE`` pins
    the choices (``ops/tuning.py``)."""

    def __init__(self):
        super().__init__("conv", "LWAAAI_GEMM_TUNE")


TUNER = ConvTuner()


def _row_default(M: int, N: int) -> int:
    if N <= 64:
        return 3 if M >= 4096 else 6
    return 2 if M * N >= (1 << 20) else 6


# ----------------------------------------------------------------------------- weight packing
def _c4_input(x: torch.Tensor) -> torch.Tensor:
    """[N, 3, H, W] → bf16 channels_last [N, 4, H, W] with a zero 4th channel."""
    x = x.to(h16())
    if x.shape[1] == 4:
        return x.contiguous(memory_format=CL)
    out = torch.zeros((x.shape[0], x.shape[2], x.shape[3], 4), dtype=h16(),
                      device=x.device).permute(0, 3, 1, 2)
    out[:, :3].copy_(x)
    return out


def pack_fwd_weight(w: torch.Tensor) -> Tuple[torch.Tensor, int, int]:
    """Weight [Co, C, R, S] → bf16 GEMM operand [Co][K] (K-contiguous). For C in (3, 4) the taps
    along w are padded to an even count and the channels to 4. Returns (operand, K, TS)."""
    co, c, r, s = w.shape
    wb = w.to(h16())
    if c % 8 == 0:
        return wb.permute(0, 2, 3, 1).contiguous().view(co, -1), r * s * c, s
    ts = s + (s & 1)
    p = torch.zeros((co, r, ts, 4), dtype=h16(), device=w.device)
    p[:, :, :s, :c].copy_(wb.permute(0, 2, 3, 1))
    return p.view(co, -1), r * ts * 4, ts


def _dgrad_classes(H, W, R, S, sh, sw, ph, pw):
    """Output-parity classes of the data gradient: (ch, cw, r0, s0, TR, TS, Hg, Wg, oh, ow)."""
    out = []
    for ch in range(sh):
        r0 = (ch + ph) % sh
        TR = len(range(r0, R, sh))
        Hg = len(range(ch, H, sh))
        for cw in range(sw):
            s0 = (cw + pw) % sw
            TS = len(range(s0, S, sw))
            Wg = len(range(cw, W, sw))
            if TR == 0 or TS == 0 or Hg == 0 or Wg == 0:
                continue                     # no tap reaches these pixels: gradient stays 0
            out.append((ch, cw, r0, s0, TR, TS, Hg, Wg, (ch + ph - r0) // sh, (cw + pw - s0) // sw))
    return out


def pack_dgrad_weight(w: torch.Tensor, classes, sh: int, sw: int,
                      fresh: bool = True) -> Tuple[torch.Tensor, List[int]]:
    """Per-class slabs Wt_c[jr][js][co][ci] = w[co, ci, r0 + sh*jr, s0 + sw*js], concatenated:
    one pack launch (``csrc/conv.hip k_pack_dgrad_nkc``) for a channels_last GPU weight, else the
    permute / slice / cat form (the reference implementation of the same layout)."""
    co, c, R, S = w.shape
    wb = w.to(h16())
    if (wb.is_cuda and c % 8 == 0 and wb.is_contiguous(memory_format=CL) and
            wb.data_ptr() % 16 == 0):
        cls, offs, off = [], [], 0
        for (_ch, _cw, r0, s0, TR, TS, *_r) in classes:
            cls += [r0, s0, TR, TS]
            offs.append(off)
            off += TR * TS * co * c
        return kc_pack(wb, cls, sh, sw, 0, fresh or wb is not w), offs
    wt = wb.permute(2, 3, 0, 1)                               # [R, S, Co, C]
    if len(classes) == 1 and classes[0][4] == R and classes[0][5] == S:
        return wt.contiguous().view(-1), [0]
    parts, offs, off = [], [], 0
    for (ch, cw, r0, s0, TR, TS, *_r) in classes:
        p = wt[r0::sh][:TR][:, s0::sw][:, :TS].reshape(-1)
        parts.append(p)
        offs.append(off)
        off += p.numel()
    return torch.cat(parts), offs


def pack_dgrad_weight_kc(w: torch.Tensor, classes, sh: int, sw: int, fresh: bool = True):
    """K-contiguous per-class slabs Wk_c[ci][jr][js][co] = w[co, ci, r0 + sh*jr, s0 + sw*js]
    (the transpose of :func:`pack_dgrad_weight`'s slabs), each row padded to the largest class K
    so that one row stride serves every class; one launch (``csrc/conv.hip k_pack_dgrad_kc``).
    Returns (packed, offsets, row stride)."""
    co, c, R, S = w.shape
    kmax = max(TR * TS * co for (_c, _w, _r, _s, TR, TS, *_x) in classes)
    kmax = -(-kmax // 8) * 8
    cls = []
    for (_c, _w, r0, s0, TR, TS, *_x) in classes:
        cls += [r0, s0, TR, TS]
    wb = w.to(h16()).contiguous(memory_format=CL)
    packed = kc_pack(wb, cls, sh, sw, kmax, fresh or wb is not w)
    return packed, [i * c * kmax for i in range(len(classes))], kmax


# ----------------------------------------------------------------------------- the three passes
def conv_fwd(x: torch.Tensor, w: torch.Tensor, stride, padding, pro=None, stats=False,
             wpack=None, bias=None, relu=False, xin=None):
    """y = conv2d(x, w) as bf16 channels_last [N, Co, Ho, Wo]; optionally the input BN-apply+ReLU
    ``pro = (scale, shift)`` (fp32 [C]), the per-M-tile column statistics of y, and an fp32
    ``bias`` [Co] / ReLU applied in the epilogue before the bf16 rounding."""
    lib = load()
    sh, sw = _pair(stride)
    ph, pw = _pair(padding)
    co, c, R, S = w.shape
    c4 = c % 8 != 0
    if xin is None:                   # (``xin``: the caller's _c4_input(x) for a C = 3/4 input)
        xin = _c4_input(x) if c4 else x.to(h16()).contiguous(memory_format=CL)
    Nb, _, H, W = xin.shape
    Ho, Wo = out_size(H, R, sh, ph), out_size(W, S, sw, pw)
    op, K, TS = wpack if wpack is not None else pack_fwd_weight(w)
    C = xin.shape[1]
    geom = [Nb, H, W, C, sh, sw, 1, 1, Ho, Wo, 1, 1, 1,
            R, TS, -ph, -pw, Ho, Wo, 0, 0, K, 0]
    mode = CV_A4 if c4 else CV_A
    ps, pt = (pro[0], pro[1]) if pro is not None else (None, None)
    M = Nb * Ho * Wo

    bf = bias.float().contiguous() if bias is not None else None

    def run(tile):
        if tile == STEM_DIRECT:               # NHWC output: as the [pixels, Co] GEMM rows
            ys, sts = lib.stem_conv7(xin, op)
            return ys.permute(0, 2, 3, 1).reshape(M, co), sts
        if tile == CONV3_TAP:
            ys, sts = lib.conv3_tap(xin, op, co, bool(stats))
            return ys.permute(0, 2, 3, 1).reshape(M, co), (sts if stats else None)
        return lib.conv_ex(xin, op, mode, geom, co, tile, 1, True, ps, pt, stats, None, False, 0,
                           True, K, bias=bf, relu=bool(relu))
    key = ("f", tuple(xin.shape), tuple(w.shape), sh, sw, ph, pw, pro is not None, stats,
           bias is not None, bool(relu))
    big = BIG_TILES if (not c4 and C % 64 == 0 and pro is None and co % 8 == 0) else ()
    direct = (STEM_DIRECT,) if (c4 and co == 64 and (R, S) == (7, 7) and
                                (sh, sw) == (2, 2) and (ph, pw) == (3, 3) and pro is None and
                                bias is None and not relu and Ho % 4 == 0 and
                                (4 * Wo) % 112 == 0 and 4 * Wo <= 448) else ()
    if (pro is None and bias is None and not relu and not c4 and
            _conv3_tap_fits(C, co, R, S, sh, sw, ph, pw, H, W)):
        direct = direct + (CONV3_TAP,)
    tile = TUNER.pick(key, run, ROW_TILES + big + direct, _row_default(M, co))
    y, st = run(tile)
    return y.view(Nb, Ho, Wo, co).permute(0, 3, 1, 2), st


def conv_dgrad(dy: torch.Tensor, w: torch.Tensor, x_hw, stride, padding, wpack=None,
               out: Optional[torch.Tensor] = None, addend: Optional[torch.Tensor] = None):
    """dx [N, C, H, W] (bf16 channels_last) of conv2d(x, w) given dy [N, Co, Ho, Wo].

    ``out`` (bf16 [N*H*W, C] rows) receives the result — only the pixels some tap reaches are
    written — and ``addend`` (same layout, may be ``out`` itself) is added to them after rounding:
    ``conv_dgrad(dy, w, hw, 2, 0, out=dx, addend=dx)`` accumulates a strided 1x1 shortcut's data
    gradient into dx in place."""
    lib = load()
    sh, sw = _pair(stride)
    ph, pw = _pair(padding)
    co, c, R, S = w.shape
    H, W = x_hw
    dyc = dy.to(h16()).contiguous(memory_format=CL)
    Nb, _, Ho, Wo = dyc.shape
    classes = _dgrad_classes(H, W, R, S, sh, sw, ph, pw)
    if not classes:
        if out is not None:
            return _nchw_rows(out, Nb, H, W)
        return torch.zeros((Nb, c, H, W), dtype=h16(), device=dy.device, memory_format=CL)
    # the [K][C] slabs are packed only if that layout runs (a "kc" / "tap" / "direct" pick packs
    # its own); their offsets are known without packing
    if wpack is not None:
        offs = wpack[1]
    else:
        offs, o = [], 0
        for (_ch, _cw, _r0, _s0, TR, TS, *_r) in classes:
            offs.append(o)
            o += TR * TS * co * c
    nkc_pack = [wpack[0] if wpack is not None else None]

    def nkc_weight(fresh):
        if nkc_pack[0] is None:
            nkc_pack[0] = pack_dgrad_weight(w, classes, sh, sw, fresh)[0]
        return nkc_pack[0]
    geom = [Nb, Ho, Wo, co, 1, 1, -1, -1, H, W, sh, sw, len(classes)]
    for (ch, cw, r0, s0, TR, TS, Hg, Wg, oh, ow), off in zip(classes, offs):
        geom += [TR, TS, oh, ow, Hg, Wg, ch, cw, TR * TS * co, off]
    M = max(Nb * cl[6] * cl[7] for cl in classes)

    def run(cand, dst=None, add=None, fresh=True):
        layout, tile = cand
        if layout == "tap" and (dst is not None or add is not None):
            layout, tile = "kc", 2            # the direct kernels write a fresh tensor only
        if layout == "tap":           # (the flip + transpose pack is timed with the conv)
            ys, _ = lib.conv3_tap(dyc, tap_dgrad_weight(w, fresh), c, False)
            return ys.permute(0, 2, 3, 1).reshape(-1, c), None
        if layout == "kc":            # (the tuner times a pack of its own with the conv)
            wk, koffs, kmax = pack_dgrad_weight_kc(w, classes, sh, sw, fresh)
            g = list(geom)
            for i, off in enumerate(koffs):
                g[13 + 10 * i + 9] = off
            return lib.conv_ex(dyc, wk, CV_A, g, c, tile, 1, True, None, None, False, dst, False,
                               0, True, kmax, add)
        return lib.conv_ex(dyc, nkc_weight(fresh), CV_A, geom, c, tile, 1, True, None, None,
                           False, dst, False, 0, False, c, add)
    key = ("d", tuple(dyc.shape), tuple(w.shape), H, W, sh, sw, ph, pw, addend is not None,
           False)
    # the weight as [K][C] (the kernel's transposing LDS reads) or packed K-contiguous [C][K]
    # (LDS-DMA staging of both operands)
    big = BIG_TILES if (len(classes) == 1 and sh == 1 and sw == 1 and co % 64 == 0 and
                        c % 8 == 0 and addend is None) else ()
    cands = [("nkc", t) for t in ROW_TILES] + [("kc", t) for t in ROW_TILES + big]
    if (addend is None and out is None and
            _conv3_tap_fits(co, c, R, S, sh, sw, ph, pw, Ho, Wo) and (H, W) == (Ho, Wo)):
        cands.append(("tap", CONV3_TAP))
    cand = TUNER.pick(key, run, cands, ("nkc", _row_default(M, c)))   # (timed on scratch outputs)
    dx, _ = run(cand, out, addend, False)
    return _nchw_rows(dx, Nb, H, W)


def _nchw_rows(rows: torch.Tensor, n: int, h: int, w: int) -> torch.Tensor:
    return rows.view(n, h, w, rows.shape[-1]).permute(0, 3, 1, 2)


def _wgrad_splits(tiles: int, pixels: int, bk: int) -> int:
    want = max(1, (2 * 256) // max(tiles, 1))
    return int(max(1, min(want, pixels // (bk * 8))))


def conv_wgrad(dy: torch.Tensor, x: torch.Tensor, w_shape, stride, padding, pro=None,
               out: Optional[torch.Tensor] = None, xin=None):
    """dW of conv2d(x, w): fp32 [Co][R][S'][C'] GEMM output. With ``out`` (a dense fp32 view of
    the weight's gradient in [Co][R][S][C] memory order, C % 8 == 0) the result is accumulated
    into it in place and ``out`` is returned; otherwise a fresh [Co, C, R, S] tensor (channels_last
    memory) is returned."""
    lib = load()
    sh, sw = _pair(stride)
    ph, pw = _pair(padding)
    co, c, R, S = w_shape
    c4 = c % 8 != 0
    if pro is not None:
        # the input's BN-apply+ReLU, materialised once (a B-gather prologue would redo it for
        # every tap and output-channel tile)
        xa = x.to(h16()).contiguous(memory_format=CL)
        x = lib.bn_apply(xa, torch.cat([pro[0][:c], pro[1][:c]]).contiguous(), None, None, True)
        pro = None
    if xin is None:
        xin = _c4_input(x) if c4 else x.to(h16()).contiguous(memory_format=CL)
    dyc = dy.to(h16()).contiguous(memory_format=CL)
    Nb, C, H, W = xin.shape
    _, _, Ho, Wo = dyc.shape
    TS = S + (S & 1) if c4 else S
    N = R * TS * C
    pix = Nb * Ho * Wo
    geom = [Nb, H, W, C, sh, sw, 1, 1, Ho, Wo, 1, 1, 1, R, TS, -ph, -pw, Ho, Wo, 0, 0, 0, 0]
    mode = CV_B4 if c4 else CV_B
    ps, pt = (pro[0], pro[1]) if pro is not None else (None, None)

    # the big tiles with the im2col column gather (csrc/gemm_big.hip GB): C % 8, Co % 8, no prologue
    big = BIG_TILES if (not c4 and co % 8 == 0 and pro is None) else ()

    def cands():
        cs = []
        for t in COL_TILES + big:
            bm, bn, bk = _TILE_DIMS[t]
            tiles = -(-co // bm) * -(-N // bn)
            s0 = _wgrad_splits(tiles, pix, bk)
            for s in sorted({max(1, s0 // 8), max(1, s0 // 4), max(1, s0 // 2), s0, s0 * 2}):
                cs.append((t, s))
        return cs

    def run(cand, dst=None, acc=False):
        t, s = cand
        if t == "tap":                # fp32 [Co][3][3][C], written into / added onto dst
            o = lib.conv3_tap_wgrad(dyc, xin, dst, acc)
            return o.permute(0, 2, 3, 1).reshape(co, -1), None
        return lib.conv_ex(xin, dyc, mode, geom, N, t, s, False, ps, pt, False, dst, acc, 0,
                           False, co)
    key = ("w", tuple(xin.shape), tuple(dyc.shape), tuple(w_shape), sh, sw, ph, pw,
           pro is not None)
    bm, bn, bk = _TILE_DIMS[1]
    default = (1, _wgrad_splits(-(-co // bm) * -(-N // bn), pix, bk))
    cs = cands()
    if pro is None and not c4 and (H, W) == (Ho, Wo) and \
            _conv3_tap_fits(C, co, R, S, sh, sw, ph, pw, H, W):
        cs.append(("tap", 0))
    cand = TUNER.pick(key, run, cs, default)
    direct = out is not None and not c4
    if direct:
        run(cand, out, True)
        return out
    g, _ = run(cand)
    g = g.view(co, R, TS, C)[:, :, :S, :c]
    return g.permute(0, 3, 1, 2)


# ----------------------------------------------------------------------------- autograd layer
def _arena_view(p: torch.Tensor):
    """The parameter's fp32 gradient-arena view when the engine wants it written in place and
    its memory order is [Co][R][S][C] (channels_last), else None."""
    if getattr(p, "_lw_grad_ready", None) is None or p.grad is None:
        return None
    g = p.grad
    if g.dtype != torch.float32 or not g.is_contiguous(memory_format=CL):
        return None
    return g


def _bias_arena_view(b: Optional[torch.Tensor]):
    """The bias's fp32 [C] gradient-arena view when the engine wants it written in place."""
    if b is None or getattr(b, "_lw_grad_ready", None) is None or b.grad is None:
        return None
    g = b.grad
    return g if g.dtype == torch.float32 and g.is_contiguous() and g.dim() == 1 else None


class _ConvFn(torch.autograd.Function):
    """conv2d (+ bias) (+ ReLU) on the implicit-GEMM kernels. Bias and ReLU run in the forward
    epilogue; backward masks dy by the saved output and reduces the bias gradient in one pass
    (``csrc/nn.hip`` k_relu_bias_bwd) before the data / weight gradient convs."""

    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, relu):
        from .block import _bf16_weight
        wb = _bf16_weight(weight)
        if weight.shape[1] % 8 != 0:
            # a 3/4-channel image: its zero-padded 4-channel copy is built once and kept for the
            # weight gradient (three launches fewer in backward)
            xs = _c4_input(x)
            y, _ = conv_fwd(x, wb, stride, padding, bias=bias, relu=relu, xin=xs)
        else:
            y, _ = conv_fwd(x, wb, stride, padding, bias=bias, relu=relu)
            xs = x.to(h16()).contiguous(memory_format=CL)
        ctx.save_for_backward(xs, wb, y if relu else None)
        ctx.geom = (stride, padding, tuple(x.shape[2:]), x.dtype)
        ctx.weight = weight
        ctx.bias = bias
        ctx.relu = relu
        return y

    @staticmethod
    def backward(ctx, dy):
        xs, wb, y = ctx.saved_tensors
        stride, padding, hw, xdtype = ctx.geom
        w, b = ctx.weight, ctx.bias
        dx = dw = db = None
        dy = dy.to(h16()).contiguous(memory_format=CL)
        if ctx.relu or (b is not None and ctx.needs_input_grad[2]):
            # an arena-managed bias gets its gradient accumulated in place by the fold kernel
            # (no AccumulateGrad add kernel, no fresh [C] buffer)
            db_dst = _bias_arena_view(b) if ctx.needs_input_grad[2] else None
            if dy.shape[1] % 8 == 0 and dy.shape[1] <= 2048:
                dy, db = load().relu_bias_bwd(dy, y if ctx.relu else None, db_dst)
                if db_dst is not None:
                    b._lw_grad_ready(b)
                    db = None
            else:
                if ctx.relu:
                    dy = dy * (y > 0)
                db = dy.float().sum((0, 2, 3))
            db = db.to(b.dtype) if db is not None and b is not None and \
                ctx.needs_input_grad[2] else None
        if ctx.needs_input_grad[0]:
            dx = conv_dgrad(dy, wb, hw, stride, padding).to(xdtype)
        if ctx.needs_input_grad[1]:
            dst = _arena_view(w)
            c4 = w.shape[1] % 8 != 0
            if dst is not None and not c4:
                conv_wgrad(dy, xs, tuple(w.shape), stride, padding, out=dst)
                w._lw_grad_ready(w)
            elif dst is not None:
                # [Co][R][TS][4] GEMM output: its [:, :, :S, :C] slice added into the arena view
                # by one strided add (no contiguous copy, no AccumulateGrad add)
                dst.add_(conv_wgrad(dy, xs, tuple(w.shape), stride, padding, xin=xs))
                w._lw_grad_ready(w)
            else:
                dw = conv_wgrad(dy, xs, tuple(w.shape), stride, padding,
                                xin=xs if c4 else None).to(w.dtype)
                dw = dw.contiguous(memory_format=CL) if w.is_contiguous(memory_format=CL) \
                    else dw.contiguous()
        return dx, dw, db, None, None, None


def mfma_conv2d(x, weight, bias=None, stride=1, padding=0, relu=False):
    """bf16 MFMA convolution (+ bias, + ReLU in the epilogue); outside autocast an fp32 input
    gets an fp32 output back."""
    y = _ConvFn.apply(x, weight, bias, _pair(stride), _pair(padding), bool(relu))
    if x.dtype == torch.float32 and not torch.is_autocast_enabled():
        y = y.float()
    return y


class MFMAConv2d(nn.Conv2d):
    """nn.Conv2d (same parameters / state_dict) on the MFMA implicit-GEMM kernels for CUDA
    inputs; CPU tensors and unsupported configurations keep the torch path."""

    def forward(self, x):
        if x.is_cuda and isinstance(self.padding, tuple) and self.padding_mode == "zeros" and \
                supported(self.in_channels, self.out_channels, self.groups, self.dilation):
            return mfma_conv2d(x, self.weight, self.bias, self.stride, self.padding,
                               getattr(self, "fuse_relu", False))
        y = super().forward(x)
        return F.relu(y) if getattr(self, "fuse_relu", False) else y


def to_mfma_conv(m: nn.Conv2d) -> nn.Conv2d:
    if type(m) is nn.Conv2d:
        m.__class__ = MFMAConv2d
    return m


def fuse_convs(model: nn.Module, relu: bool = True) -> nn.Module:
    """Switch every plain nn.Conv2d of ``model`` to :class:`MFMAConv2d` (in place; parameter and
    buffer names are unchanged, so checkpoints stay compatible). With ``relu``, a Conv2d directly
    followed by a ReLU inside an nn.Sequential (VGG / AlexNet features) gets the ReLU in its
    epilogue and the ReLU module becomes an Identity."""
    if relu:
        for mod in model.modules():
            if isinstance(mod, nn.Sequential):
                kids = list(mod._modules.items())
                for i, (name, child) in enumerate(kids):
                    if type(child) is nn.Conv2d and i + 1 < len(kids) and \
                            isinstance(kids[i + 1][1], nn.ReLU):
                        to_mfma_conv(child)
                        child.fuse_relu = True
                        mod._modules[kids[i + 1][0]] = nn.Identity()
                        # a max-pool right after the ReLU: the ReLU-aware pool kernels
                        if i + 2 < len(kids) and type(kids[i + 2][1]) is nn.MaxPool2d:
                            from .nn import ReluMaxPool2d
                            kids[i + 2][1].__class__ = ReluMaxPool2d
    for m in model.modules():
        if type(m) is nn.Conv2d:
            to_mfma_conv(m)
    return model
