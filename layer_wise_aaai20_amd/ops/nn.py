"""Model-path ops backed by the HIP kernels of ``csrc/nn.hip`` (GPU) or torch (CPU)."""
from __future__ import annotations

import torch
from torch import nn

from ._ext import ops_for


def normalize_nhwc_u8(images: torch.Tensor, mean: torch.Tensor, std: torch.Tensor,
                      dtype=torch.bfloat16) -> torch.Tensor:
    """uint8 [N, H, W, C] → ``(x - mean) / std`` as an NCHW tensor in channels_last memory.

    One fused pass on the GPU; the reference does collate → ``.cuda()`` →
    ``.half()`` → ``sub_`` → ``div_`` (``IMAGENET/training/dataloader.py:81-93``)."""
    assert images.dtype == torch.uint8 and images.dim() == 4
    N, H, W, C = images.shape
    lib = ops_for(images)
    if lib is not None and images.is_contiguous():
        out = torch.empty((N, C, H, W), dtype=dtype, device=images.device,
                          memory_format=torch.channels_last)
        lib.normalize_u8(images, out, [float(m) for m in mean.tolist()],
                         [float(s) for s in std.tolist()])
        return out
    x = images.permute(0, 3, 1, 2).float()
    x = (x - mean.view(1, -1, 1, 1).to(x.device)) / std.view(1, -1, 1, 1).to(x.device)
    return x.to(dtype).contiguous(memory_format=torch.channels_last)


def fuse_resnet(model: nn.Module) -> nn.Module:
    """Hook for swapping BN/ReLU/residual chains for fused HIP kernels (kept as a no-op until the
    fused kernels beat the library path on MI355X; see profiles/)."""
    return model
