"""Dump the gradient and residual the entire-model Top-K codec sees on a real CIFAR AlexNet step
(BASELINE config 3), as raw little-endian float32 files for scripts/probes/select_probe.hip
(`select_probe N K iters 0 g.f32 e.f32`). Eager steps; the last step's pair is written."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--out", default="gpurun_out/em_grad")
    a = ap.parse_args()
    from layer_wise_aaai20_amd.train.cifar_fast import CifarTrainer
    tr = CifarTrainer("alexnet", device="cuda", compress="entiremodel", method="Topk", K=0.01,
                      error_feedback=True, n_train=512 * 8, graph=False)
    eng = tr.ddp.engine
    codec = eng.codecs[0]
    real = codec.compress
    seen = {}

    def capture(g, ef, step):
        seen["g"] = g.detach().clone()
        seen["e"] = ef.detach().clone() if ef is not None else torch.zeros_like(g)
        return real(g, ef, step)
    codec.compress = capture
    for _ in range(a.steps):
        tr.step()
    torch.cuda.synchronize()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    seen["g"].float().cpu().numpy().tofile(a.out + "_g.f32")
    seen["e"].float().cpu().numpy().tofile(a.out + "_e.f32")
    g = seen["g"].float()
    print({"n": g.numel(), "zeros": int((g == 0).sum()), "absmax": float(g.abs().max())})


if __name__ == "__main__":
    main()
