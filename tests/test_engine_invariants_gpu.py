"""Bucket-launch invariants on the real fused MI355X paths (SURVEY.md §5 race detection): with
``GradSyncEngine._check`` on, every gradient segment must be announced exactly once per step and
never after its bucket was launched — the fused ops write gradients straight into the arena and
announce them, and PyTorch then also runs their post-accumulate-grad hooks
(profiles/r2_vgg_fault.md). Runs a few steps of ResNet-50 (block path) and CIFAR VGG-16 (MFMA
convs / linears) with compression overlapped on the side stream and the fused SGD."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_resnet50_block_path_invariants(monkeypatch):
    from layer_wise_aaai20_amd.train.imagenet import build_trainer
    torch.manual_seed(0)
    tr = build_trainer("resnet50", device="cuda", compress="layerwise", method="Topk", K=0.001)
    eng = tr.ddp.engine
    monkeypatch.setattr(eng, "_check", True)
    launches = []
    real = eng._launch
    monkeypatch.setattr(eng, "_launch", lambda bi: (launches.append(bi), real(bi)))
    for _ in range(3):
        launches.clear()
        x = torch.randint(0, 256, (16, 64, 64, 3), dtype=torch.uint8, device="cuda")
        t = torch.randint(0, 1000, (16,), device="cuda")
        tr.step(x, t)
        assert launches == list(range(len(eng.buckets)))
    torch.cuda.synchronize()
    assert all(eng._marked)


def test_vgg16_mfma_path_invariants(monkeypatch):
    from layer_wise_aaai20_amd.models.cifar import build_network
    from layer_wise_aaai20_amd.ops.conv import fuse_convs
    from layer_wise_aaai20_amd.ops.gemm import fuse_linears
    from layer_wise_aaai20_amd.optim.flat_sgd import FlatSGD
    from layer_wise_aaai20_amd.parallel.ddp import CompressedDDP
    torch.manual_seed(0)
    net = build_network("vgg16")
    fuse_convs(net)
    fuse_linears(net)
    net = net.cuda().to(memory_format=torch.channels_last)
    ddp = CompressedDDP(net, compress="layerwise", method="Topk", K=0.001, flat_params=True)
    monkeypatch.setattr(ddp.engine, "_check", True)
    opt = FlatSGD(list(net.parameters()), ddp.arena, lr=1e-3, momentum=0.9, nesterov=True)
    x = torch.randn(64, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (64,), device="cuda")
    for _ in range(4):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = ddp({"input": x, "target": y})
        out["loss"].float().sum().backward()
        opt.step()
        assert all(ddp.engine._marked)
    torch.cuda.synchronize()
