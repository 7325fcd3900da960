"""Stage-by-stage graph-vs-eager bisection of the CIFAR trainer step.

Runs the same training twice in one process — eager (reference) and with the HIP-graph step — plus
an eager control run, and records for every step and every bucket, through copies into persistent
buffers issued on the codec's own stream (so they are captured into the graph too):

  g_in   gradient bucket before compression      e_in   error-feedback residual before
  send   compressed payload                      e_out  residual after
  idx    (Random-K index-free) selected indices  g_out  decoded bucket
  param  flat parameters after the step          x      the step's input batch (static copy)

and prints, per step, the first stage at which the graph run departs from the eager run.

argv: network mode method [K] [steps] [flags...]
flags: force (capture codecs kept eager), torchaug (torch gather augmentation), noauto (no
graph-vs-eager timing decision), overlap0 (LWAAAI_OVERLAP=0).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
args = sys.argv[1:]
flags = set(a for a in args[3:] if not a.replace(".", "").isdigit())
nums = [a for a in args[3:] if a.replace(".", "").isdigit()]
if "overlap0" in flags:
    os.environ["LWAAAI_OVERLAP"] = "0"
if "noauto" in flags:
    os.environ["LWAAAI_GRAPH_AUTO"] = "0"
os.environ.setdefault("LWAAAI_GRAPH_ENTIRE", "1")

import torch  # noqa: E402
from layer_wise_aaai20_amd.compress import codecs as C  # noqa: E402
from layer_wise_aaai20_amd.train.cifar_fast import CifarTrainer  # noqa: E402
from layer_wise_aaai20_amd.utils.logging import PiecewiseLinear  # noqa: E402

net, mode, method = args[:3]
K = float(nums[0]) if nums else 0.05
STEPS = int(nums[1]) if len(nums) > 1 else 10
if "force" in flags:
    C.RandkSparseCodec.graph_safe = True

STAGES = ("x", "g_in", "e_in", "ws", "send", "idx", "e_out", "g_out", "param")


def instrument(tr):
    """Wrap every codec of the trainer's engine with stage copies into persistent buffers."""
    eng = tr.ddp.engine
    dbg = {}

    def buf(key, like):
        t = dbg.get(key)
        if t is None or t.shape != like.shape or t.dtype != like.dtype:
            assert not torch.cuda.is_current_stream_capturing(), f"new debug buffer {key} in capture"
            t = torch.empty_like(like)
            dbg[key] = t
        return t

    def cp(dst, src):
        # kcopy: an elementwise kernel instead of a D2D memcpy (a memcpy node inside a graph)
        if "kcopy" in flags:
            torch.mul(src, 1, out=dst)
        else:
            dst.copy_(src)

    for bi, codec in enumerate(eng.codecs):
        comp, decomp = codec.compress, codec.decompress

        def compress(grad, ef, step, bi=bi, comp=comp, codec=codec):
            cp(buf(("g_in", bi), grad), grad)
            if ef is not None:
                cp(buf(("e_in", bi), ef), ef)
            out = comp(grad, ef, step)
            cp(buf(("send", bi), out), out)
            idx = getattr(codec, "_idx", {}).get(str(grad.device))
            if idx is not None:
                cp(buf(("idx", bi), idx), idx)
            if ef is not None:
                cp(buf(("e_out", bi), ef), ef)
            ws = getattr(codec, "_ws", {}).get(str(grad.device))
            if ws is not None:
                cp(buf(("ws", bi), ws), ws)
            return out

        def decompress(send, recv, grad, world=None, bi=bi, decomp=decomp):
            decomp(send, recv, grad, world)
            cp(buf(("g_out", bi), grad), grad)

        codec.compress, codec.decompress = compress, decompress
    return dbg


def run(graph: bool, tag: str):
    torch.manual_seed(0)
    tr = CifarTrainer(net, compress=mode, method=method, K=K, error_feedback=method != "none",
                      batch_size=128, epochs=2, n_train=6400, seed=0, graph=graph)
    if "torchaug" in flags:
        tr.batches.use_kernel = False
    tr.steps_per_epoch = 1
    tr.sched = PiecewiseLinear([0, 40, 200], [0, 0.4, 0])
    dbg = instrument(tr)
    hist = []
    for i in range(STEPS):
        b = tr.next_batch()
        if "syncbatch" in flags:
            torch.cuda.synchronize()
        loss = float(tr.step(b))
        torch.cuda.synchronize()
        snap = {k: v.detach().float().cpu().clone() for k, v in dbg.items()}
        snap[("x", 0)] = b["input"].float().cpu().clone()
        snap[("param", 0)] = tr.ddp.arena.param_buf.detach().float().cpu().clone()
        hist.append((loss, snap))
    g = tr.graphed
    print(f"[{tag}] graph enabled={g.enabled} replays={g.replays} decided={g.decided} "
          f"losses " + " ".join(f"{h[0] / tr.bs:.4f}" for h in hist), flush=True)
    return hist


def compare(a, b, name):
    print(f"== {name}", flush=True)
    for i, ((la, sa), (lb, sb)) in enumerate(zip(a, b)):
        first = None
        parts = []
        for st in STAGES:
            for key in sorted(k for k in sa if k[0] == st):
                if key not in sb:
                    continue
                d = float((sa[key] - sb[key]).abs().max()) if sa[key].numel() else 0.0
                neq = int((sa[key] != sb[key]).sum())
                if d != 0 or neq:
                    parts.append(f"{st}{key[1]}:{d:.2e}/{neq}")
                    if first is None:
                        first = f"{st}[{key[1]}]"
        zeros = ""
        if ("e_out", 0) in sa and ("e_out", 0) in sb:
            zeros = (f" e_out zeros {int((sa[('e_out', 0)] == 0).sum())}/"
                     f"{int((sb[('e_out', 0)] == 0).sum())}")
        print(f"step {i}: loss {la:.6f}/{lb:.6f} first={first}{zeros} " + " ".join(parts),
              flush=True)
        if first is not None and ("ws", 0) in sa and not getattr(compare, "shown", False):
            compare.shown = True
            for tag, s in (("A", sa), ("B", sb)):
                print(f"  {tag}: {decode_ws(s[('ws', 0)])}", flush=True)


def decode_ws(wsf, n_tasks=None):
    """Entire-model Top-K workspace (one large segment): hist | st_small | st_large | cnt | pre."""
    import numpy as np
    b = wsf.to(torch.uint8).numpy()
    hist = b[0:16384].view(np.uint32)
    st = b[16640:16640 + 32].view(np.uint32)
    nt = n_tasks or (6573120 + 8191) // 8192
    cnt_off = 16896
    cnt = b[cnt_off:cnt_off + 8 * nt].view(np.uint32).reshape(-1, 2)
    pre_off = cnt_off + (8 * nt + 255) // 256 * 256
    pre = b[pre_off:pre_off + 8 * nt].view(np.uint32).reshape(-1, 2)
    return (f"hist sums p0={hist[:2048].sum()} p1={hist[2048:3072].sum()} "
            f"p2={hist[3072:].sum()} | st prefix={st[0]:#x} m={st[1]} tkey={st[2]:#x} "
            f"quota={st[3]} gt={st[4]} total={st[5]} cap={st[6]} | cnt sum gt={cnt[:, 0].sum()} "
            f"eq={cnt[:, 1].sum()} | pre last={pre[-1].tolist()} first={pre[:3].tolist()}")


eager = run(False, "eager")
control = run(False, "eager-control")
graphed = run(True, "graph")
compare(eager, control, "eager vs eager-control")
compare(eager, graphed, "eager vs graph")
