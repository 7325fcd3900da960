#!/usr/bin/env python
"""Headline benchmark: ImageNet ResNet-50 training with layer-wise Top-K (k = 0.1 %) gradient
compression, data-parallel over N MI355X GPUs (one process per GPU, RCCL over xGMI).

BASELINE.json metric: "images/sec/node + top-1 acc, ResNet-50 Top-K k=0.1% layer-wise at 1/2/4/8
GPUs". The reference (``IMAGENET/training/train_imagenet_nv.py:388-478``) measures the same step:
forward, cross-entropy, backward, layer-wise Top-K compression + gradient exchange, SGD step.

What one timed step does here (nothing skipped):
  uint8 synthetic batch -> fused normalise to bf16 NHWC -> ResNet-50 forward/backward (bf16
  autocast, channels_last) -> per-bucket HIP Top-K select + pack overlapped with backward ->
  RCCL all-gather of (index, value) pairs -> rank-ordered unpack/average -> fused SGD (Nesterov,
  momentum 0.9, wd 1e-4 with BN excluded) over the flat parameter arena.

Usage:
  python bench.py                                   # 1 GPU
  torchrun --nproc-per-node 8 bench.py --gpus 8     # one node
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))


def _miopen_cache_env() -> None:
    """Point MIOpen's find-db and compiled-kernel cache at an in-repo directory (unless the user
    already chose one): the solver search and kernel compilation of a fresh box then run once per
    image, not once per run (a cold find for ResNet-50 takes minutes)."""
    base = os.path.join(ROOT, ".miopen")
    for var, sub in (("MIOPEN_USER_DB_PATH", "db"), ("MIOPEN_CUSTOM_CACHE_DIR", "cache")):
        if var not in os.environ:
            path = os.path.join(base, sub)
            os.makedirs(path, exist_ok=True)
            os.environ[var] = path


_miopen_cache_env()

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

BASELINE_METRIC = ("images/sec/node + top-1 acc, ResNet-50 Top-K k=0.1% layer-wise at "
                   "1/2/4/8 GPUs")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--compress", default="layerwise")
    ap.add_argument("--method", default="Topk")
    ap.add_argument("--ratio", "-K", type=float, default=0.001)
    ap.add_argument("--threshold", "-V", type=float, default=0.001)
    ap.add_argument("--qstates", "-Q", type=int, default=255)
    ap.add_argument("--ef", action="store_true", help="error feedback")
    ap.add_argument("--bucket-mb", type=float, default=25.0)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-fused", action="store_true", help="disable fused HIP nn kernels")
    ap.add_argument("--json-out", default="")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend (nccl = RCCL on ROCm)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="debug: every rank on cuda:0 (multi-rank plumbing on a 1-GPU box, gloo)")
    ap.add_argument("--miopen-find", type=int, default=1,
                    help="1: let MIOpen benchmark conv solvers once (cudnn.benchmark)")
    return ap.parse_args()


class _Heartbeat:
    """Progress on stderr every 20 s while warm-up runs (MIOpen's first solver search can take
    minutes with no output)."""

    def __init__(self, rank: int, every: float = 20.0):
        import threading
        self.rank, self.msg, self.t0 = rank, "warmup 0", time.time()
        self._stop = threading.Event()
        self._th = threading.Thread(target=self._run, args=(every,), daemon=True)
        self._th.start()

    def _run(self, every):
        while not self._stop.wait(every):
            if self.rank == 0:
                print(f"[bench] {self.msg} ({time.time() - self.t0:.0f} s)", file=sys.stderr,
                      flush=True)

    def note(self, msg: str) -> None:
        self.msg = msg

    def stop(self) -> None:
        self._stop.set()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    if args.share_gpu:
        local = 0
    torch.cuda.set_device(local)
    torch.backends.cudnn.benchmark = bool(args.miopen_find)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    from layer_wise_aaai20_amd.train.imagenet import build_trainer

    tr = build_trainer(model=args.model, device=dev, compress=args.compress, method=args.method,
                       K=args.ratio, V=args.threshold, qstates=args.qstates,
                       error_feedback=args.ef, bucket_cap_mb=args.bucket_mb, dtype=args.dtype,
                       fused=not args.no_fused, momentum=0.9, weight_decay=1e-4, no_bn_wd=True,
                       lr=0.1)
    B, S = args.batch, args.image_size
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    images = torch.randint(0, 256, (B, S, S, 3), dtype=torch.uint8, device=dev, generator=g)
    target = torch.randint(0, 1000, (B,), device=dev, generator=g)

    beat = _Heartbeat(rank)
    for i in range(args.warmup):
        tr.step(images, target)
        beat.note(f"warmup {i + 1}/{args.warmup}")
    beat.stop()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.step(images, target)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    top1 = tr.last_top1()
    ms = dt / args.steps * 1e3
    value = world * B * args.steps / dt
    stats = tr.ddp.sync_stats()
    default = (args.model == "resnet50" and args.compress == "layerwise" and args.method == "Topk"
               and args.ratio == 0.001)
    metric = BASELINE_METRIC if default else (
        f"images/sec/node, {args.model} {args.compress} {args.method}"
        f"{' K=' + str(args.ratio) if args.method in ('Topk', 'Randomk') else ''}"
        f"{' +EF' if args.ef else ''}")
    line = {
        "metric": metric,
        "value": round(value, 2),
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (random uint8 224x224 images, random labels; random-init weights)",
        "top1_train_synthetic": round(top1, 3) if top1 is not None else None,
        "config": {
            "model": args.model,
            "global_batch": world * B,
            "per_gpu_batch": B,
            "image_size": S,
            "seq_len": None,
            "parallelism": f"dp{world}",
            "compress": args.compress,
            "method": args.method,
            "ratio": args.ratio,
            "error_feedback": args.ef,
            "wire_bytes_per_rank": stats.payload_bytes,
            "dense_grad_bytes": stats.dense_bytes,
            "buckets": stats.buckets,
        },
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                json.dump(line, f)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
