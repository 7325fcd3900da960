"""relu_pool forward/backward on a small map with the device-resident identity constants, checked
against torch (prints the max error; a HIP error surfaces as a RuntimeError with its text)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from layer_wise_aaai20_amd.ops._ext import load  # noqa: E402

lib = load()
x = torch.relu(torch.randn(2, 64, 8, 8, device="cuda")).bfloat16().contiguous(
    memory_format=torch.channels_last)
out, idx = lib.relu_pool_fwd(x, 2, 2, 0)
ref = torch.nn.functional.max_pool2d(x.float(), 2, 2)
print("fwd max err", float((out.float() - ref).abs().max()), flush=True)
dp = torch.randn_like(out)
dx = lib.relu_pool_bwd(dp.contiguous(memory_format=torch.channels_last), idx, x, 2, 2, 0)
xr = x.float().requires_grad_()
torch.nn.functional.max_pool2d(xr, 2, 2).backward(dp.float())
print("bwd max err", float((dx.float() - xr.grad * (x.float() > 0)).abs().max()), flush=True)
