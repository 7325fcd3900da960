"""Decode fused with the SGD step (parallel/engine.py set_fused_sgd,
csrc/compress.hip k_unpack_sgd): a layer-wise Top-K bucket's averaged gradient goes from the
decode's LDS chunk straight into the optimizer update. The parameters, momentum buffers and bf16
mirror must equal those of the separate decode + FlatSGD passes bit for bit — eagerly through the
engine, and through a HIP-graph-captured CIFAR trainer step (LR read from device memory)."""
import os

import pytest
import torch
from torch import nn

from layer_wise_aaai20_amd.parallel.engine import GradSyncEngine

pytestmark = pytest.mark.gpu


def _setup(fused, nesterov, wd, mode="layerwise"):
    from layer_wise_aaai20_amd.optim.flat_sgd import FlatSGD
    torch.manual_seed(0)
    net = nn.Sequential(nn.Conv2d(16, 64, 3), nn.BatchNorm2d(64), nn.ReLU(), nn.Flatten(),
                        nn.Linear(64 * 6 * 6, 300), nn.ReLU(), nn.Linear(300, 10)).cuda()
    eng = GradSyncEngine(list(net.named_parameters()), mode=mode, method="Topk", K=0.01,
                         error_feedback=True, flat_params=True, bucket_cap_mb=0.5)
    params = list(net.parameters())
    opt = FlatSGD([{"params": params[:3], "weight_decay": 0.0},
                   {"params": params[3:], "weight_decay": wd}], eng.arena, lr=0.05,
                  momentum=0.9, nesterov=nesterov)
    eng.arena.refresh_bf16()              # the bf16 mirror both paths write along with p
    n = eng.set_fused_sgd(opt) if fused else (opt.exclude_segments(()) or 0)
    return eng, opt, n


@pytest.mark.parametrize("mode", ["layerwise", "entiremodel"])
@pytest.mark.parametrize("nesterov", [False, True])
@pytest.mark.parametrize("wd", [0.0, 5e-3])
def test_fused_decode_sgd_matches_separate_passes(nesterov, wd, mode):
    ea, oa, na = _setup(False, nesterov, wd, mode)
    eb, ob, nb = _setup(True, nesterov, wd, mode)
    assert na == 0 and nb == len(eb.buckets) >= 1
    assert nb > 1 or mode == "entiremodel"
    torch.manual_seed(1)
    for step in range(4):
        g = torch.randn(ea.arena.numel, device="cuda")
        for eng, opt in ((ea, oa), (eb, ob)):
            opt.param_groups[0]["lr"] = opt.param_groups[1]["lr"] = 0.05 / (step + 1)
            eng.arena.grad.copy_(g)
            eng.sync_now()
            opt.step()
        torch.cuda.synchronize()
        for name, a, b in (("param", ea.arena.param_buf, eb.arena.param_buf),
                           ("momentum", oa.buf, ob.buf), ("ef", ea.ef, eb.ef),
                           ("bf16", ea.arena.param_bf16, eb.arena.param_bf16)):
            assert torch.equal(a, b), (step, name, (a - b).abs().max().item())


def test_cifar_graph_step_fused_sgd_bitwise():
    from layer_wise_aaai20_amd.train.cifar_fast import CifarTrainer
    outs = []
    for flag in ("0", "1"):
        torch.manual_seed(0)                        # (the same initial weights for both runs)
        tr = CifarTrainer(device="cuda", n_train=512 * 6, graph=True, network="resnet9",
                          compress="layerwise", method="Topk", K=0.01, error_feedback=True,
                          seed=0, fused_sgd=flag == "1")
        tr.graphed.warmup = 2
        fused = len(tr.ddp.engine._sgd_buckets)
        assert (fused > 0) == (flag == "1")
        for _ in range(6):
            tr.step()
        torch.cuda.synchronize()
        assert tr.graphed.replays >= 2
        outs.append((tr.ddp.arena.param_buf.clone(), tr.opt.buf.clone()))
        del tr
    (pa, ba), (pb, bb) = outs
    assert torch.equal(pa, pb), (pa - pb).abs().max().item()
    assert torch.equal(ba, bb)


def test_vgg_claimed_overwrite_matches_zero_and_accumulate():
    """VGG-16's fc1 weight gradient is written by one copy into an arena slice the step did not
    zero (engine.claim_overwrite) instead of zero + add: the trained parameters equal the
    zero-and-accumulate path's (engine.CLAIM_OVERWRITE = False), graph-captured steps included."""
    from layer_wise_aaai20_amd.parallel import engine as E
    from layer_wise_aaai20_amd.train.cifar_fast import CifarTrainer
    outs = []
    for flag in ("0", "1"):
        E.CLAIM_OVERWRITE = flag == "1"
        torch.manual_seed(0)
        try:
            tr = CifarTrainer(device="cuda", n_train=512 * 6, graph=True, network="vgg16",
                              compress="layerwise", method="Topk", K=0.001, seed=0)
            tr.graphed.warmup = 2
            for _ in range(6):
                tr.step()
            torch.cuda.synchronize()
            if flag == "1":
                assert tr.ddp.engine._no_zero, "fc1 should be written by a claimed overwrite"
            outs.append(tr.ddp.arena.param_buf.clone())
        finally:
            E.CLAIM_OVERWRITE = True
        del tr
    assert torch.equal(outs[0], outs[1]), (outs[0] - outs[1]).abs().max().item()
