"""Notebook analysis toolkit (utils/analysis.py): functional optimisers, label smoothing,
Hessian-vector products."""
import numpy as np
import torch
from torch import nn

from layer_wise_aaai20_amd.models.graph import Network, union
from layer_wise_aaai20_amd.utils import analysis as A


def test_nesterov_update_matches_torch_sgd():
    torch.manual_seed(0)
    w0 = torch.randn(50)
    grads = [torch.randn(50) for _ in range(5)]
    w = w0.clone().requires_grad_()
    opt = A.SGD_fn([w], {"lr": lambda s: 0.1, "weight_decay": lambda s: 5e-4,
                         "momentum": lambda s: 0.9})
    ref = w0.clone().requires_grad_()
    topt = torch.optim.SGD([ref], lr=0.1, momentum=0.9, nesterov=True, weight_decay=5e-4)
    for g in grads:
        w.grad = g.clone()
        opt = A.opt_step(**opt)
        ref.grad = g.clone()
        topt.step()
    torch.testing.assert_close(w.detach(), ref.detach(), rtol=1e-5, atol=1e-6)
    assert opt["step_number"] == 5


def test_lars_scales_by_trust_ratio():
    w = torch.full((4,), 2.0)
    dw = torch.full((4,), 0.5)
    v = torch.zeros(4)
    A.LARS_update(w, dw.clone(), v, lr=0.1, weight_decay=0.0, momentum=0.0)
    ratio = 4.0 / (1.0 + 1e-2)                   # |w| = 4, |dw| = 1
    torch.testing.assert_close(w, torch.full((4,), 2.0 - 0.1 * ratio * 0.5))


def test_label_smoothing_losses_match_torch():
    torch.manual_seed(1)
    net = Network(union({"classifier": {"out": nn.Linear(8, 5)}},
                        A.losses(alpha=0.8, beta=0.2)))
    x, t = torch.randn(16, 8), torch.randint(0, 5, (16,))
    out = net({"input": x, "target": t})
    ref = nn.functional.cross_entropy(out["classifier_out"], t, label_smoothing=0.2,
                                      reduction="none")
    torch.testing.assert_close(out["loss"], ref, rtol=1e-5, atol=1e-6)
    assert out["correct"].shape == (16,)


class _Quad(nn.Module):
    def __init__(self, a):
        super().__init__()
        self.register_buffer("a", torch.tensor(a))
        self.w = nn.Parameter(torch.ones(len(a)))

    def forward(self, batch):
        return {"loss": (0.5 * self.a * self.w ** 2 * batch).sum().reshape(1)}


def test_hessian_top_eigens_of_quadratic():
    m = _Quad([3.0, 1.0, 7.0, 0.5])
    op = A.HvOperator(m, [torch.tensor(1.0), torch.tensor(1.0)])
    vals, vecs = A.compute_top_k_eigens(op, 2, tol=1e-8)
    np.testing.assert_allclose(vals, [7.0, 3.0], rtol=1e-5)
    assert abs(abs(vecs[0][2]) - 1.0) < 1e-4


def test_perturbed_model_and_vectors():
    m = nn.Linear(3, 2)
    vec = torch.arange(8, dtype=torch.float32)
    p = A.perturbed_model(m, vec)
    torch.testing.assert_close(A.to_vec(p.parameters()) - A.to_vec(m.parameters()), vec)
    basis = A.orthogonal_subspace(np.eye(4)[:1])
    assert basis.shape == (3, 4) and np.allclose(basis @ np.eye(4)[0], 0)
    x = torch.randn(1000)
    y = A.ShiftScaleReLU()(x)           # the notebook's constants (cell 43)
    torch.testing.assert_close(y, (torch.relu(x) - (1 / np.pi) ** 0.5) / (1 - 1 / np.pi) ** 0.5)
