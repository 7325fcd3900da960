"""Dict-defined network graphs (the cifar10-fast API the reference's CIFAR code is built on).

API-compatible re-implementation of ``CIFAR10/core.py:121-141`` (``union``, ``path_iter``,
``rel_path``, ``build_graph``) and ``CIFAR10/torch_backend.py:69-143`` (layer nodes, ``Network``,
``trainable_params``, ``TorchOptimiser``, ``SGD``). A network is a nested dict whose leaves are
modules (input = the previous node) or ``(module, [input paths])`` tuples; ``Network`` flattens it
into an insertion-ordered DAG and ``forward`` returns the dict of every node's output, so the loss
and accuracy are nodes too.
"""
from __future__ import annotations

from collections import namedtuple
from typing import Callable, Dict, Iterable

import torch
from torch import nn

sep = "_"
RelativePath = namedtuple("RelativePath", ("parts",))


def rel_path(*parts) -> RelativePath:
    return RelativePath(parts)


def union(*dicts) -> dict:
    out = {}
    for d in dicts:
        out.update(d)
    return out


def path_iter(nested: dict, pfx=()):
    for name, val in nested.items():
        if isinstance(val, dict):
            yield from path_iter(val, (*pfx, name))
        else:
            yield (*pfx, name), val


def _resolve(path, pfx) -> str:
    if isinstance(path, RelativePath):
        return sep.join((*pfx, *path.parts))
    if isinstance(path, str):
        return path
    return sep.join(path)


def build_graph(net: dict) -> Dict[str, tuple]:
    """``{name: (module, [input names])}``; a bare module's input is the previous node
    (``'input'`` for the first), matching ``core.py:136-141``."""
    flat = list(path_iter(net))
    graph = {}
    prev = "input"
    for (*pfx, name), val in flat:
        key = sep.join((*pfx, name))
        if isinstance(val, tuple):
            mod, inputs = val
            graph[key] = (mod, [_resolve(i, pfx) for i in inputs])
        else:
            graph[key] = (val, [prev])
        prev = key
    return graph


class Identity(nn.Module):
    def forward(self, x):
        return x


class Mul(nn.Module):
    def __init__(self, weight):
        super().__init__()
        self.weight = weight

    def forward(self, x):
        return x * self.weight


class Flatten(nn.Module):
    def forward(self, x):
        return x.reshape(x.size(0), x.size(1))


class Add(nn.Module):
    def forward(self, x, y):
        return x + y


class Concat(nn.Module):
    def forward(self, *xs):
        return torch.cat(xs, 1)


class Correct(nn.Module):
    def forward(self, classifier, target):
        return classifier.max(dim=1)[1] == target


def batch_norm(num_channels, bn_bias_init=None, bn_bias_freeze=False, bn_weight_init=None,
               bn_weight_freeze=False) -> nn.BatchNorm2d:
    m = nn.BatchNorm2d(num_channels)
    with torch.no_grad():
        if bn_bias_init is not None:
            m.bias.fill_(bn_bias_init)
        if bn_weight_init is not None:
            m.weight.fill_(bn_weight_init)
    m.bias.requires_grad_(not bn_bias_freeze)
    m.weight.requires_grad_(not bn_weight_freeze)
    return m


class Network(nn.Module):
    """Executes a ``build_graph`` DAG; ``forward(inputs: dict) -> dict of all node outputs``."""

    def __init__(self, net: dict):
        super().__init__()
        self.graph = build_graph(net)
        for name, (mod, _) in self.graph.items():
            self.add_module(name, mod)

    def forward(self, inputs: dict) -> dict:
        cache = dict(inputs)
        for name, (_, ins) in self.graph.items():
            cache[name] = self._modules[name](*[cache[i] for i in ins])
        # (the reference keeps the live dict, torch_backend.py:69-80; a detached view keeps the
        # outputs inspectable without holding the previous step's autograd graph — and its
        # AccumulateGrad nodes — alive into the next step, which breaks HIP-graph capture)
        self.cache = {k: (v.detach() if torch.is_tensor(v) else v) for k, v in cache.items()}
        return cache


def trainable_params(model: nn.Module) -> Iterable[nn.Parameter]:
    return filter(lambda p: p.requires_grad, model.parameters())


class TorchOptimiser:
    """Optimizer whose hyper-parameters may be callables of the step number
    (``torch_backend.py:124-140``): re-evaluated and pushed into the param group every ``step``."""

    def __init__(self, weights, optimizer: Callable, step_number: int = 0, **opt_params):
        self.weights = weights
        self.step_number = step_number
        self.opt_params = opt_params
        self._opt = optimizer(weights, **self.param_values())

    def param_values(self) -> dict:
        return {k: v(self.step_number) if callable(v) else v for k, v in self.opt_params.items()}

    def step(self):
        self.step_number += 1
        vals = self.param_values()
        for g in self._opt.param_groups:
            g.update(**vals)
        self._opt.step()

    def zero_grad(self, set_to_none: bool = True):
        self._opt.zero_grad(set_to_none=set_to_none)

    def state_dict(self):
        return self._opt.state_dict()

    def load_state_dict(self, sd):
        self._opt.load_state_dict(sd)

    @property
    def param_groups(self):
        return self._opt.param_groups

    def __repr__(self):
        return repr(self._opt)


def SGD(weights, lr=0, momentum=0, weight_decay=0, dampening=0, nesterov=False,
        optimizer: Callable = torch.optim.SGD) -> TorchOptimiser:
    return TorchOptimiser(weights, optimizer, lr=lr, momentum=momentum,
                          weight_decay=weight_decay, dampening=dampening, nesterov=nesterov)
