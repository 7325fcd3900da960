"""Mixed-precision helpers with the reference API (``IMAGENET/training/fp16util.py``): an fp16 (or
bf16) model whose BatchNorm layers stay fp32, fp32 master weights (optionally one flat tensor),
and grad/param copies between them; static loss scaling is applied by the training loop
(``train_imagenet_nv.py:411-428``).

On MI355X the default training path is bf16 autocast with fp32 parameters (no loss scale needed);
these helpers keep ``--fp16`` runs of the reference recipe working.
"""
from __future__ import annotations

import torch
from torch import nn
from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors


class tofp16(nn.Module):
    def forward(self, x):
        return x.half()


def BN_convert_float(module: nn.Module) -> nn.Module:
    """Keep BatchNorm in fp32 (cuDNN/MIOpen fp16 BN wants fp32 parameters)."""
    if isinstance(module, nn.modules.batchnorm._BatchNorm):
        module.float()
    for child in module.children():
        BN_convert_float(child)
    return module


def network_to_half(network: nn.Module, dtype=torch.float16) -> nn.Module:
    """``nn.Sequential(tofp16(), BN_convert_float(network.half()))`` (fp16util.py:32-43)."""
    cast = tofp16() if dtype == torch.float16 else _ToDtype(dtype)
    return nn.Sequential(cast, BN_convert_float(network.to(dtype)))


class _ToDtype(nn.Module):
    def __init__(self, dtype):
        super().__init__()
        self.dtype = dtype

    def forward(self, x):
        return x.to(self.dtype)


def prep_param_lists(model: nn.Module, flat_master: bool = False):
    """(model_params, master_params) with fp32 masters (fp16util.py:49-88)."""
    model_params = [p for p in model.parameters() if p.requires_grad]
    if flat_master:
        master = _flatten_dense_tensors([p.data.float() for p in model_params])
        master = nn.Parameter(master)
        master.grad = master.new_zeros(master.size())
        return model_params, [master]
    master_params = [p.detach().clone().float() for p in model_params]
    for p in master_params:
        p.requires_grad = True
    return model_params, master_params


def model_grads_to_master_grads(model_params, master_params, flat_master: bool = False):
    if flat_master:
        master_params[0].grad.data.copy_(_flatten_dense_tensors(
            [p.grad.data for p in model_params]))
        return
    for m, mp in zip(model_params, master_params):
        if m.grad is None:
            mp.grad = None
            continue
        if mp.grad is None:
            mp.grad = torch.empty_like(mp)
        mp.grad.data.copy_(m.grad.data)


def master_params_to_model_params(model_params, master_params, flat_master: bool = False):
    if flat_master:
        for m, mp in zip(model_params, _unflatten_dense_tensors(master_params[0].data,
                                                                  model_params)):
            m.data.copy_(mp)
        return
    for m, mp in zip(model_params, master_params):
        m.data.copy_(mp.data)


def backwards_debug_hook(grad):
    raise RuntimeError("master_params received a gradient in the backward pass!")
