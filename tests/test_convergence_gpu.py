"""Convergence smoke: ResNet-9 on the class-conditional synthetic CIFAR-10
(``data/cifar.py synthetic_cifar10``: a per-class colour offset under noise), trained through the
full MI355X path — fused graph net, MFMA convs / linear, CompressedDDP, FlatSGD — for ~200 steps
with every compression method in both granularities, error feedback on. Recipe of
``CIFAR10/dawn.py:98-155`` (summed loss, per-sample LR from the piecewise-linear schedule,
Nesterov momentum, wd 5e-4·bs) at a shorter horizon. The loss must fall and held-out accuracy
must beat chance (10 %) by a wide margin. Accuracy parity with the reference's real-data runs
is unpinned (no CIFAR-10 here).

Error feedback needs a contractive compressor (||C(v) - v||² < ||v||²). QSGD with s levels on an
n-element vector has relative variance up to sqrt(n)/s: ≈ 20 for s = 127 over the whole
6.6 M-parameter ResNet-9 and ≈ 12 for its largest layer, so with EF the residual grows
geometrically (entire-model: the loss reached 1e14 in 200 steps on MI355X; layer-wise: held-out
accuracy 25 %). QSGD therefore runs with 16-bit codes here (s = 32767, variance ≈ 0.08); the 8/9-bit
codes are checked bit for bit against the CPU mirror in tests/test_kernels_gpu.py."""
import pytest
import torch

pytestmark = pytest.mark.gpu

METHODS = [("none", {}), ("Topk", {"K": 0.01}), ("Randomk", {"K": 0.05}),
           ("Thresholdv", {"V": 1e-3}), ("AdaptiveThreshold", {}), ("TernGrad", {}),
           ("RandomDithering", {"qstates": 32767})]


@pytest.mark.parametrize("mode", ["layerwise", "entiremodel"])
@pytest.mark.parametrize("method,kw", METHODS, ids=[m for m, _ in METHODS])
def test_resnet9_learns_with_compression(method, kw, mode):
    from layer_wise_aaai20_amd.data import cifar as D
    from layer_wise_aaai20_amd.train.cifar_fast import CifarTrainer
    torch.manual_seed(0)
    tr = CifarTrainer("resnet9", compress=mode if method != "none" else "none", method=method,
                      error_feedback=method != "none", batch_size=128, epochs=2,
                      n_train=12800, seed=0, task="colour", **kw)
    from layer_wise_aaai20_amd.utils.logging import PiecewiseLinear
    steps = 200
    tr.steps_per_epoch = 1                           # schedule in steps: warm-up 40, decay to 0
    # entire-model TernGrad scales the ternary code by max|g| over all 6.6 M parameters, so its
    # variance dwarfs ||g||²: at the recipe's peak LR it diverges without EF (loss 2.8e26 over 24
    # epochs, profiles/r3/cifar_method_accuracy_table.jsonl) and can stall with it (loss 1.02 ->
    # 1.05 on one tuner draw); it trains at a quarter of the peak LR
    peak = 0.1 if (method, mode) == ("TernGrad", "entiremodel") else 0.4
    tr.sched = PiecewiseLinear([0, 40, steps], [0, peak, 0])
    losses = []
    for _ in range(steps):
        losses.append(float(tr.step()) / tr.bs)
    first, last = sum(losses[:20]) / 20, sum(losses[-20:]) / 20
    assert all(l == l for l in losses), "NaN loss"
    assert last < first * 0.8, (first, last)
    # held-out accuracy on fresh samples of the same synthetic distribution
    ds = D.synthetic_cifar10(16, 2048, seed=1, task="colour")["test"]
    x = torch.from_numpy(D.transpose(D.normalise(ds["data"]))).cuda()
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.as_tensor(ds["labels"]).cuda()
    tr.model.eval()
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        out = tr.model({"input": x, "target": y})
    acc = float(out["correct"].float().mean())
    assert acc > 0.3, acc
