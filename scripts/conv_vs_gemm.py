"""Micro-benchmark: MIOpen 1x1 conv (NHWC bf16) vs hipBLASLt GEMM on the same data, for the
ResNet-50 1x1 shapes at batch 256 / 224 px. fwd, dgrad, wgrad timed separately."""
import torch
import torch.nn.functional as F

torch.backends.cudnn.benchmark = True
dev = "cuda"
B = 256
shapes = [  # (H, Cin, Cout)
    (56, 64, 64), (56, 64, 256), (56, 256, 64), (28, 128, 512), (28, 512, 128),
    (14, 256, 1024), (14, 1024, 256), (7, 512, 2048), (7, 2048, 512),
]


def bench(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


tot = {"conv": 0.0, "gemm": 0.0}
for H, ci, co in shapes:
    x = torch.randn(B, ci, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(co, ci, 1, 1, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(B, co, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    M = B * H * H
    x2 = x.permute(0, 2, 3, 1).reshape(M, ci)
    dy2 = dy.permute(0, 2, 3, 1).reshape(M, co)
    w2 = w.reshape(co, ci)
    flops = 2 * M * ci * co
    cf = bench(lambda: F.conv2d(x, w))
    cd = bench(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [True, False, False]))
    cw = bench(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False]))
    gf = bench(lambda: torch.mm(x2, w2.t()))
    gd = bench(lambda: torch.mm(dy2, w2))
    gw = bench(lambda: torch.mm(dy2.t(), x2))
    tot["conv"] += cf + cd + cw
    tot["gemm"] += gf + gd + gw
    tf = lambda t: flops / t / 1e9
    print(f"H{H:3d} {ci:5d}->{co:5d}  conv f/d/w {cf:6.3f} {cd:6.3f} {cw:6.3f} ms ({tf(cf):5.0f}/{tf(cd):5.0f}/{tf(cw):5.0f} TF)"
          f"   gemm f/d/w {gf:6.3f} {gd:6.3f} {gw:6.3f} ms ({tf(gf):5.0f}/{tf(gd):5.0f}/{tf(gw):5.0f} TF)", flush=True)
print(tot)
