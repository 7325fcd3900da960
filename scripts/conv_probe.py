"""One 1x1-conv forward shape through MIOpen and through the MFMA GEMM (for counter collection).
usage: conv_probe.py H Cin Cout tile [batch]"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from layer_wise_aaai20_amd.ops import gemm as G  # noqa: E402

torch.backends.cudnn.benchmark = True
H, ci, co = (int(v) for v in sys.argv[1:4])
tile = sys.argv[4]
B = int(sys.argv[5]) if len(sys.argv) > 5 else 256
x = torch.randn(B, ci, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
w = torch.randn(co, ci, 1, 1, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
M = B * H * H
x2 = x.permute(0, 2, 3, 1).reshape(M, ci)
w2 = w.reshape(co, ci)
for _ in range(5):
    F.conv2d(x, w)
    G.gemm_ex(x2, ci, True, w2, ci, True, M, co, ci, tile=tile)
torch.cuda.synchronize()
