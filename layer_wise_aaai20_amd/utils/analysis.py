"""Experiment / analysis toolkit of the reference's CIFAR notebooks.

``CIFAR10/batch_norm_post.ipynb`` bundles a newer cifar10-fast library for its BatchNorm study;
its reusable pieces are provided here on top of this package's graph API
(:mod:`..models.graph`):

* functional optimisers — ``nesterov_update`` / ``LARS_update`` with the ``optimiser`` /
  ``opt_step`` / ``opt_steps`` state-dict style driver (notebook cell 8);
* label-smoothing losses — ``losses(alpha, beta)`` graph nodes ``logp → KL, xent → loss =
  alpha·xent + beta·KL`` (cells 8, 61);
* ``ShiftScaleReLU`` (cell 43), channel statistics ``channel_vars`` / ``channel_skews``
  (cell 124), ``orthogonal_subspace`` (cell 122);
* curvature — flat parameter vectors, ``perturbed_model``, ``compute_grad`` (gradient or
  Hessian/Jacobian-vector product averaged over fixed batches) and ``HvOperator`` +
  ``compute_top_k_eigens`` (Lanczos via ``scipy.sparse.linalg.eigsh``; cell 109).

Everything is plain PyTorch (these are offline analysis tools, not the training hot path); on an
MI355X the Hessian-vector products run through the same autograd graph as training.
"""
from __future__ import annotations

import copy
import math
import time
from collections import namedtuple
from functools import partial
from itertools import count
from typing import Callable, Dict, Iterable, List, Optional, Sequence

import numpy as np
import torch
from torch import nn

from ..models.graph import Correct

__all__ = ["nesterov_update", "LARS_update", "zeros_like", "optimiser", "opt_step", "opt_steps",
           "SGD_fn", "LARS", "LogSoftmax", "KLLoss", "CrossEntropyLoss", "AddWeighted", "losses",
           "ShiftScaleReLU", "to_vec", "named_trainable", "param_dict_from_vec",
           "perturbed_model", "compute_grad", "loss_grad", "HvOperator", "compute_top_k_eigens",
           "channel_vars", "channel_skews", "orthogonal_subspace"]


# ----------------------------------------------------------------------------- optimisers
@torch.no_grad()
def nesterov_update(w, dw, v, lr, weight_decay, momentum):
    """In place: ``dw ← -lr(dw + wd·w)``; ``v ← momentum·v + dw``; ``w += dw + momentum·v``."""
    dw.add_(w, alpha=weight_decay).mul_(-lr)
    v.mul_(momentum).add_(dw)
    w.add_(dw.add_(v, alpha=momentum))


@torch.no_grad()
def LARS_update(w, dw, v, lr, weight_decay, momentum):
    """Nesterov step with the layer-wise trust ratio ``‖w‖ / (‖dw‖ + 1e-2)`` scaling the LR."""
    ratio = (w.norm() / (dw.norm() + 1e-2)).to(w.dtype)
    nesterov_update(w, dw, v, lr * ratio, weight_decay, momentum)


def zeros_like(weights: Sequence[torch.Tensor]) -> List[torch.Tensor]:
    return [torch.zeros_like(w) for w in weights]


def optimiser(weights, param_schedule: Dict[str, Callable[[int], float]], update,
              state_init) -> dict:
    weights = list(weights)
    return {"update": update, "param_schedule": param_schedule, "step_number": 0,
            "weights": weights, "state": state_init(weights)}


def opt_step(update, param_schedule, step_number, weights, state) -> dict:
    step_number += 1
    values = {k: f(step_number) for k, f in param_schedule.items()}
    for w, v in zip(weights, state):
        if w.requires_grad and w.grad is not None:
            update(w.data, w.grad.data, v, **values)
    return {"update": update, "param_schedule": param_schedule, "step_number": step_number,
            "weights": weights, "state": state}


def opt_steps(optimisers: Iterable[dict]) -> List[dict]:
    return [opt_step(**o) for o in optimisers]


SGD_fn = partial(optimiser, update=nesterov_update, state_init=zeros_like)
LARS = partial(optimiser, update=LARS_update, state_init=zeros_like)


# ----------------------------------------------------------------------------- losses
class LogSoftmax(nn.Module):
    def __init__(self, dim: int = 1):
        super().__init__()
        self.dim = dim

    def forward(self, x):
        return torch.log_softmax(x.float(), self.dim)


class KLLoss(nn.Module):
    """KL to the uniform distribution up to a constant: ``-mean_c log p_c`` per sample."""

    def forward(self, log_probs):
        return -log_probs.mean(dim=1)


class CrossEntropyLoss(nn.Module):
    """Per-sample NLL of log-probabilities (``reduction='none'``)."""

    def forward(self, log_probs, target):
        return nn.functional.nll_loss(log_probs, target, reduction="none")


class AddWeighted(nn.Module):
    def __init__(self, wx: float, wy: float):
        super().__init__()
        self.wx, self.wy = wx, wy

    def forward(self, x, y):
        return self.wx * x + self.wy * y


def losses(alpha: Optional[float] = None, beta: Optional[float] = None,
           logits: str = "classifier_out") -> dict:
    """Loss nodes for a dict-graph network: plain cross-entropy (``alpha is None``) or label
    smoothing ``alpha·xent + beta·KL(uniform)``; ``correct`` is always added."""
    if alpha is None:
        return {"loss": (nn.CrossEntropyLoss(reduction="none"), [logits, "target"]),
                "correct": (Correct(), [logits, "target"])}
    return {"logp": (LogSoftmax(1), [logits]),
            "KL": (KLLoss(), ["logp"]),
            "xent": (CrossEntropyLoss(), ["logp", "target"]),
            "loss": (AddWeighted(alpha, beta), ["xent", "KL"]),
            "correct": (Correct(), [logits, "target"])}


class ShiftScaleReLU(nn.Module):
    """ReLU re-centred and re-scaled to zero mean / unit variance for N(0,1) inputs."""

    def forward(self, x):
        return (torch.relu(x) - math.sqrt(1.0 / math.pi)) * (1.0 / math.sqrt(1.0 - 1.0 / math.pi))


# ----------------------------------------------------------------------------- curvature
def named_trainable(model: nn.Module) -> Dict[str, torch.Tensor]:
    return {k: p for k, p in model.named_parameters() if p.requires_grad}


def to_vec(tensors: Iterable[torch.Tensor]) -> torch.Tensor:
    return torch.cat([t.reshape(-1) for t in tensors])


def param_dict_from_vec(vec, template: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    out, off = {}, 0
    for k, p in template.items():
        out[k] = vec[off: off + p.numel()].reshape(p.shape)
        off += p.numel()
    return out


def perturbed_model(model: nn.Module, vec) -> nn.Module:
    """A deep copy of ``model`` with ``vec`` (flat, trainable-parameter order) added to its
    parameters; buffers are copied unchanged."""
    vec = torch.as_tensor(vec)
    delta = param_dict_from_vec(vec, named_trainable(model))
    clone = copy.deepcopy(model)
    with torch.no_grad():
        for k, p in clone.named_parameters():
            if k in delta:
                p.add_(delta[k].to(device=p.device, dtype=p.dtype))
    return clone


def compute_grad(model: nn.Module, batches: Sequence, outputs: Callable, vec=None) -> torch.Tensor:
    """Mean over ``batches`` of ∂outputs(model, batch)/∂params (flat fp32), contracted with
    ``vec`` as ``grad_outputs`` when given (vector-Jacobian / Hessian-vector products)."""
    params = list(named_trainable(model).values())
    total = None
    for batch in batches:
        out = outputs(model, batch)
        g = torch.autograd.grad(out, params, grad_outputs=vec, allow_unused=True)
        g = to_vec(torch.zeros_like(p) if gi is None else gi for gi, p in zip(g, params)).float()
        total = g if total is None else total + g
    return total / len(batches)


def loss_grad(model: nn.Module, batch) -> torch.Tensor:
    """Flat gradient of the summed loss with ``create_graph`` (differentiable again)."""
    params = list(named_trainable(model).values())
    out = model(batch)["loss"].sum()
    return to_vec(torch.autograd.grad(out, params, create_graph=True))


try:
    import scipy.sparse.linalg as _sla

    class HvOperator(_sla.LinearOperator):
        """Hessian of the summed training loss over fixed batches as a scipy LinearOperator
        (each matvec = one Hessian-vector product through double backward)."""

        def __init__(self, model: nn.Module, batches: Sequence, projection=None):
            self.model, self.batches, self.projection = model, batches, projection
            params = list(named_trainable(model).values())
            n = int(sum(p.numel() for p in params))
            self.torch_dtype = params[0].dtype
            self.device = params[0].device
            self.iterations = count(1)
            self.log: List[dict] = []
            self._t0 = time.time()
            super().__init__(dtype=np.dtype("float32"), shape=(n, n))

        def _matvec(self, v):
            v = torch.as_tensor(np.asarray(v).reshape(-1), dtype=self.torch_dtype,
                                device=self.device)
            hv = compute_grad(self.model, self.batches, loss_grad, v).cpu().numpy()
            self.log.append({"iteration": next(self.iterations),
                             "total time": time.time() - self._t0})
            return self.projection(hv) if self.projection else hv

    def compute_top_k_eigens(op, k: int, tol: float = 1e-4):
        """Largest-k eigenpairs (descending) by Lanczos."""
        vals, vecs = _sla.eigsh(A=op, k=k, tol=tol, return_eigenvectors=True)
        return vals[::-1], vecs.T[::-1]
except ImportError:  # pragma: no cover - scipy is part of the image
    HvOperator = None
    compute_top_k_eigens = None


# ----------------------------------------------------------------------------- statistics
def channel_vars(model: nn.Module, batch, node: str = "classifier_out") -> torch.Tensor:
    return model(batch)[node].var(0)


def channel_skews(model: nn.Module, batch, node: str = "classifier_out") -> torch.Tensor:
    logits = model(batch)[node]
    return ((logits - logits.mean(0, keepdim=True)) ** 3).mean(0)


def orthogonal_subspace(vecs: np.ndarray) -> np.ndarray:
    """Orthonormal basis of the orthogonal complement of span(rows of ``vecs``)."""
    vecs = np.atleast_2d(np.asarray(vecs, dtype=np.float64))
    _, s, vt = np.linalg.svd(vecs, full_matrices=True)
    rank = int((s > s.max(initial=0.0) * 1e-10).sum()) if s.size else 0
    return vt[rank:]
