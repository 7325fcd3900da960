"""Per-op roofline of one eager ResNet-50 training step (bs 256, 224 px, layer-wise Top-K): every
GEMM / convolution / BatchNorm / pooling call of the fused path is bracketed by HIP events on the
compute stream and priced against max(FLOP / dense bf16 peak, minimum bytes / HBM rate). Prints
the calls sorted by the time they spend above that floor, then totals per kind.

usage: python scripts/op_roofline.py [--peak-tf 2300] [--hbm-tbs 6.3] [--top 40]
(the engine's side stream is dropped so compression does not interleave with the events.)"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from layer_wise_aaai20_amd.ops import _ext  # noqa: E402
from layer_wise_aaai20_amd.ops import block as blk  # noqa: E402
from layer_wise_aaai20_amd.ops import nn as lwnn  # noqa: E402
from layer_wise_aaai20_amd.train.imagenet import build_trainer  # noqa: E402

REC = []


def _pair(v):
    return tuple(v) if isinstance(v, (list, tuple)) else (v, v)
ON = [False]


def _nbytes(v):
    if isinstance(v, torch.Tensor):
        return v.numel() * v.element_size()
    if isinstance(v, (list, tuple)):
        return sum(_nbytes(u) for u in v)
    return 0


def _bracket(kind, desc, flops, fn, args, kw, extra_bytes=None):
    if not ON[0]:
        return fn(*args, **kw)
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    out = fn(*args, **kw)
    e1.record()
    nb = extra_bytes if extra_bytes is not None else _nbytes(list(args) + list(kw.values())) + \
        _nbytes(out)
    REC.append((kind, desc, flops, nb, e0, e1))
    return out


def wrap_gemm(fn):
    def g(A, lda, a_kc, B, ldb, b_kc, M, N, K, **kw):
        ob = kw.get("out_bf16", True)
        nb = 2 * (M * K + N * K) + M * N * (2 if ob else 4)
        if kw.get("accumulate"):
            nb += M * N * 4
        if kw.get("addend") is not None:
            nb += M * N * 2
        if kw.get("bst") is not None:
            nb += M * N * 2
        role = "wgrad" if kw.get("split_k") else ("fwd" if b_kc else "dgrad")
        was = ON[0]
        if not was:                        # nested calls (gemm_dgrad -> gemm) count once
            return fn(A, lda, a_kc, B, ldb, b_kc, M, N, K, **kw)
        ON[0] = False
        try:
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            e0.record()
            out = fn(A, lda, a_kc, B, ldb, b_kc, M, N, K, **kw)
            e1.record()
        finally:
            ON[0] = was
        REC.append((f"gemm-{role}", f"M{M} N{N} K{K} akc{int(a_kc)} bkc{int(b_kc)}"
                    f"{' stats' if kw.get('stats') else ''}{' pro' if kw.get('pro') else ''}",
                    2 * M * N * K, nb, e0, e1))
        return out
    return g


def wrap_dgrad(fn):
    def g(dy, ldy, W, M, N, K, **kw):
        was = ON[0]
        if not was:
            return fn(dy, ldy, W, M, N, K, **kw)
        nb = 2 * (M * K + N * K) + M * N * 2 + (M * N * 2 if kw.get("addend") is not None else 0)
        ON[0] = False
        try:
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            e0.record()
            out = fn(dy, ldy, W, M, N, K, **kw)
            e1.record()
            REC.append(("gemm-dgrad", f"M{M} N{N} K{K} (1x1 dgrad)", 2 * M * N * K, nb, e0, e1))
            return out
        finally:
            ON[0] = was
    return g


def wrap_conv(kind, fn):
    def g(*args, **kw):
        was = ON[0]
        if not was:
            return fn(*args, **kw)
        ON[0] = False
        try:
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            e0.record()
            out = fn(*args, **kw)
            e1.record()
        finally:
            ON[0] = was
        o = out[0] if isinstance(out, tuple) else out
        if kind == "conv-fwd":
            x, w = args[0], args[1]
            y = o
            cout, cin, r, s = w.shape
        elif kind == "conv-dgrad":
            y, w = args[0], args[1]
            x = o
            cout, cin, r, s = w.shape
        else:
            y, x = args[0], args[1]
            cout, cin, r, s = args[2]
        n, _, ho, wo = y.shape
        flops = 2 * n * ho * wo * cout * cin * r * s
        nb = (x.numel() + y.numel()) * 2 + cout * cin * r * s * (4 if kind == "conv-wgrad" else 2)
        st = _pair(args[2] if kind == "conv-fwd" else args[3])
        REC.append((kind, f"x{tuple(x.shape)} w{(cout, cin, r, s)} s{st[0]}", flops, nb, e0, e1))
        return out
    return g


class LibProxy:
    def __init__(self, lib, tag):
        self._lib, self._tag = lib, tag

    def __getattr__(self, name):
        f = getattr(self._lib, name)
        if not callable(f):
            return f

        def g(*a, **k):
            if not ON[0]:
                return f(*a, **k)
            shp = next((tuple(v.shape) for v in a if isinstance(v, torch.Tensor)), ())
            return _bracket(f"{self._tag}:{name}", f"{shp}", 0, f, a, k)
        return g


def _time(fn, n=20):
    fn()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n * 1e-3


def blas_compare(rows):
    """hipBLASLt (torch.matmul, bf16 in, bf16 / fp32 out) on every distinct 1x1 GEMM shape."""
    import re
    seen = {}
    for ex, t, fl, kind, desc, flops, nb in rows:
        if not kind.startswith("gemm"):
            continue
        m = re.match(r"M(\d+) N(\d+) K(\d+)", desc)
        key = (kind, desc)
        seen.setdefault(key, [t, 0, tuple(int(v) for v in m.groups())])
        seen[key][1] += 1
    print("\n1x1 GEMMs vs hipBLASLt (torch.matmul): ours_us blas_us ratio  x calls")
    dev = torch.device("cuda", 0)
    tot_o = tot_b = 0.0
    for (kind, desc), (t, cnt, (M, N, K)) in sorted(seen.items(), key=lambda x: -x[1][0] * x[1][1]):
        akc = "akc1" in desc or "dgrad" in desc
        bkc = "bkc1" in desc
        r = lambda *sh: torch.randn(*sh, device=dev, dtype=torch.bfloat16)  # noqa: E731
        a = r(M, K) if akc else r(K, M).t()      # the same operand layouts as our call
        b = r(N, K).t() if bkc else r(K, N)
        tb = _time(lambda: torch.mm(a, b))
        tot_o += t * cnt
        tot_b += tb * cnt
        print(f"  {kind:10s} {desc:40s} {t * 1e6:8.1f} {tb * 1e6:8.1f} {t / tb:5.2f}  x{cnt}")
        del a, b
    print(f"  total ours {tot_o * 1e3:.3f} ms, blas {tot_b * 1e3:.3f} ms")


def miopen_compare(rows):
    """MIOpen (torch conv, cudnn.benchmark find) on every distinct convolution call."""
    import re
    import torch.nn.functional as F
    torch.backends.cudnn.benchmark = True
    seen = {}
    for ex, t, fl, kind, desc, flops, nb in rows:
        if kind.startswith("conv"):
            seen.setdefault((kind, desc), [t, 0])[1] += 1
    print("\nconvolutions vs MIOpen: ours_us miopen_us ratio  x calls")
    dev = torch.device("cuda", 0)
    tot_o = tot_m = 0.0
    for (kind, desc), (t, cnt) in sorted(seen.items(), key=lambda x: -x[1][0] * x[1][1]):
        nums = [int(v) for v in re.findall(r"-?\d+", desc)]
        n, c, h, w = nums[0:4]
        co, ci, r, _ = nums[4:8]
        st = nums[8]
        pad = r // 2
        x = torch.randn(n, ci, h, w, device=dev, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        wt = torch.randn(co, ci, r, r, device=dev, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y = F.conv2d(x, wt, None, st, pad)
        g = torch.randn_like(y)
        if kind == "conv-fwd":
            fn = lambda: F.conv2d(x, wt, None, st, pad)  # noqa: E731
        else:
            mask = [kind == "conv-dgrad", kind == "conv-wgrad", False]
            fn = lambda: torch.ops.aten.convolution_backward(  # noqa: E731
                g, x, wt, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1, mask)
        try:
            tm = _time(fn, 10)
        except RuntimeError as e:          # noqa: PERF203
            print(f"  {kind:10s} {desc}: MIOpen failed ({str(e)[:60]})")
            continue
        tot_o += t * cnt
        tot_m += tm * cnt
        print(f"  {kind:10s} {desc:52s} {t * 1e6:8.1f} {tm * 1e6:8.1f} {t / tm:5.2f}  x{cnt}")
    print(f"  total ours {tot_o * 1e3:.3f} ms, MIOpen {tot_m * 1e3:.3f} ms")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peak-tf", type=float, default=2300.0)
    ap.add_argument("--hbm-tbs", type=float, default=6.3)
    ap.add_argument("--top", type=int, default=45)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--all", default="", help="write every call (launch order) to this file")
    ap.add_argument("--blas", action="store_true",
                    help="also time each 1x1 GEMM shape with torch.matmul (hipBLASLt)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = _ext.load()
    proxy = LibProxy(lib, "lib")
    blk.load = lambda: proxy
    lwnn.load = lambda *x, **k: proxy
    blk.gemm = wrap_gemm(blk.gemm)
    blk.gemm_dgrad = wrap_dgrad(blk.gemm_dgrad)
    blk.conv_fwd = wrap_conv("conv-fwd", blk.conv_fwd)
    blk.conv_dgrad = wrap_conv("conv-dgrad", blk.conv_dgrad)
    blk.conv_wgrad = wrap_conv("conv-wgrad", blk.conv_wgrad)
    from layer_wise_aaai20_amd.ops import conv as lwconv
    for nm in ("conv_fwd", "conv_dgrad", "conv_wgrad"):   # the stem imports these at call time
        setattr(lwconv, nm, wrap_conv(nm.replace("_", "-"), getattr(lwconv, nm)))
    tr = build_trainer("resnet50", device=dev, compress="layerwise", method="Topk", K=0.001,
                       graph=False)
    tr.ddp.engine._side = None          # compression inline: no side stream between the events
    B = a.batch
    imgs = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=dev)
    tgt = torch.randint(0, 1000, (B,), device=dev)
    for _ in range(4):
        tr.step(imgs, tgt)
    torch.cuda.synchronize()
    s0, s1 = torch.cuda.Event(True), torch.cuda.Event(True)
    s0.record()
    ON[0] = True
    tr.step(imgs, tgt)
    ON[0] = False
    s1.record()
    torch.cuda.synchronize()
    step = s0.elapsed_time(s1)
    rows = []
    for kind, desc, flops, nb, e0, e1 in REC:
        t = e0.elapsed_time(e1) * 1e-3
        floor = max(flops / (a.peak_tf * 1e12), nb / (a.hbm_tbs * 1e12))
        rows.append((t - floor, t, floor, kind, desc, flops, nb))
    tot = sum(r[1] for r in rows)
    print(f"eager step {step:.2f} ms; bracketed ops {tot * 1e3:.2f} ms over {len(rows)} calls; "
          f"floor {sum(r[2] for r in rows) * 1e3:.2f} ms (peak {a.peak_tf} TF/s, {a.hbm_tbs} TB/s)")
    print(f"{'excess_us':>9} {'t_us':>8} {'floor_us':>8} {'TF/s':>6} {'GB/s':>6}  kind  desc")
    for ex, t, fl, kind, desc, flops, nb in sorted(rows, key=lambda r: -r[0])[:a.top]:
        print(f"{ex * 1e6:9.1f} {t * 1e6:8.1f} {fl * 1e6:8.1f} {flops / t / 1e12:6.0f} "
              f"{nb / t / 1e9:6.0f}  {kind:12s} {desc}")
    if a.all:
        with open(a.all, "w") as f:
            for ex, t, fl, kind, desc, flops, nb in rows:
                f.write(f"{ex * 1e6:9.1f} {t * 1e6:8.1f} {fl * 1e6:8.1f} {flops / t / 1e12:6.0f} "
                        f"{nb / t / 1e9:6.0f}  {kind:12s} {desc}\n")
    if a.blas:
        blas_compare(rows)
        miopen_compare(rows)
    agg = collections.defaultdict(lambda: [0.0, 0.0, 0])
    for ex, t, fl, kind, *_ in rows:
        agg[kind][0] += t
        agg[kind][1] += fl
        agg[kind][2] += 1
    print("\nper kind: time / floor (ms), calls")
    for k, (t, fl, n) in sorted(agg.items(), key=lambda x: -x[1][0]):
        print(f"  {k:28s} {t * 1e3:7.3f} {fl * 1e3:7.3f}  x{n}")


if __name__ == "__main__":
    main()
