"""Diagnose CPU-mirror vs k_dequant_shard differences (QSGD): where and by how much."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import numpy as np
from layer_wise_aaai20_amd.compress import codecs
from layer_wise_aaai20_amd.compress.plan import SegPlan

sizes = [64, 3, 1000, 4096, 4097, 9408, 65536]
offs, o = [], 0
for n in sizes:
    offs.append(o)
    o += (n + 63) // 64 * 64
plan, N = SegPlan(offs, sizes), o
W = 5
for q in (127, 255):
    cs = [codecs.make_codec("QSGD", plan, W, r, qstates=q, wire="qrs", seed=9) for r in range(W)]
    g = torch.Generator().manual_seed(0)
    pays = [c.compress(torch.randn(N, generator=g) * 1e-2, None, 3).clone() for c in cs]
    r = 0
    c = cs[r]
    r1 = torch.zeros(W * c.wpr[r], dtype=torch.int32)
    rows = r1.view(W, -1)
    for p in range(W):
        for d, x in zip(c.piece_slots(rows[p], r), c.pieces(pays[p], r)):
            d.copy_(x)
    ic = torch.zeros(c.n, dtype=torch.bfloat16)
    ig = torch.zeros(c.n, dtype=torch.bfloat16, device="cuda")
    c.reduce_shard(r1, r, ic)
    c.reduce_shard(r1.cuda(), r, ig)
    ig = ig.cpu()
    d = (ic.float() - ig.float())
    bad = (ic != ig).nonzero().flatten()
    print(f"q={q} shard0 elements {c.A[1]-c.A[0]} mismatches {bad.numel()} maxdiff {d.abs().max():.3e}")
    for i in bad[:8].tolist():
        print("   idx", i, "cpu", float(ic[i]), "gpu", float(ig[i]))
    # the fp32 all-gather decodes (k_dequant vs CPU)
    ag = codecs.make_codec("QSGD", plan, W, 0, qstates=q, wire="sparse", seed=9)
    oc = torch.zeros(N)
    og = torch.zeros(N, device="cuda")
    ag.decompress(None, torch.cat(pays), oc, world=W)
    ag.decompress(None, torch.cat(pays).cuda(), og, world=W)
    print(f"   all-gather decode fp32 mismatches {(oc != og.cpu()).sum().item()} maxdiff {(oc-og.cpu()).abs().max():.3e}")
