#!/usr/bin/env python
"""Headline benchmark: ImageNet ResNet-50 training with layer-wise Top-K (k = 0.1 %) gradient
compression, data-parallel over N MI355X GPUs (one process per GPU, RCCL over xGMI).

BASELINE.json metric: "images/sec/node + top-1 acc, ResNet-50 Top-K k=0.1% layer-wise at 1/2/4/8
GPUs". The reference (``IMAGENET/training/train_imagenet_nv.py:388-478``) measures the same step:
forward, cross-entropy, backward, layer-wise Top-K compression + gradient exchange, SGD step.

What one timed step does here (nothing skipped). The whole step is one captured HIP graph
(train/graphs.py StepGraph), replayed once per step:
  uint8 synthetic batch -> fused normalise to bf16 NHWC -> ResNet-50 forward/backward (bf16,
  channels_last, hand-written MFMA / BN kernels) -> as each gradient bucket (reverse layer order)
  completes during backward: HIP Top-K select + pack, RCCL all-gather of
  (index, value) pairs, rank-ordered unpack/average fused with the SGD update (Nesterov, momentum
  0.9, wd 1e-4 with BN excluded) of that bucket's slice of the flat parameter arena.
Inside the graph a bucket's compress + collective + decode run inline on the compute stream, in
backward order, between the layers' kernels (LWAAAI_GRAPH_OVERLAP=0, parallel/engine.py): a side
stream branch per bucket ("1") measured slower under the wire-priced world-8 simulation
(README "Overlap of the exchange"; profiles/r6/sim8_wire_*_overlap_modes.jsonl). At world 1 the
exchange is a no-op and decode+SGD still run. Eager steps (no graph) do overlap the exchange on a
side stream. --simulate-world W replays the exchange of W ranks on one GPU (parallel/loopback.py) and
--sim-wire adds the modelled xGMI transfer time as CU-holding busy kernels.

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
    ap.add_argument("--ef-dense-below", type=int, default=0,
                    help="opt-in EF variant: tensors of at most this many elements sent densely")
    ap.add_argument("--momentum-correction", action="store_true",
                    help="opt-in EF variant: DGC momentum correction (profiles/r4/ef_root_cause.md)")
    # 50 MB: 3 buckets for ResNet-50's 97.5 MiB fp32 arena. Inside a captured step each bucket is
    # compressed + exchanged inline, so fewer buckets = fewer launches / collectives: 24.29 ms
    # vs 24.47-24.50 ms at the reference's 25 MB (profiles/r2_bucket_mb_graph.log)
    ap.add_argument("--bucket-mb", type=float, default=50.0)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"],
                    help="fp16: the fp16 build of the MFMA kernels with a static loss scale 1024")
    ap.add_argument("--no-fused", action="store_true", help="disable fused HIP nn kernels")
    ap.add_argument("--json-out", default="")
    ap.add_argument("--pool", type=int, default=4, help="distinct synthetic batches cycled")
    ap.add_argument("--acc-steps", type=int, default=1000,
                    help="after the timed run: train a fresh ResNet-50 with the same compression "
                         "this many steps at 128 px and report its held-out top-1 "
                         "(train/accuracy.py); 0 = not measured")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend (nccl = RCCL on ROCm)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="debug: every rank on cuda:0 (multi-rank rehearsal on a 1-GPU box; with "
                         "--backend nccl each rank declares its own RCCL host id, so the native "
                         "communicator, captured collectives and teardown run as on a node)")
    ap.add_argument("--simulate-world", type=int, default=0,
                    help="time a world of W ranks on this one GPU (train/simworld.py: codecs, "
                         "decode and captured side-stream branch for W ranks, loopback "
                         "communicator with replayed peer payloads) and print one JSON line per "
                         "configuration instead of the benchmark line")
    ap.add_argument("--sim-wire", action="store_true",
                    help="with --simulate-world: every collective also pays its modelled xGMI "
                         "transfer time as a busy kernel (parallel/loopback.py WireModel)")
    ap.add_argument("--sim-overlap", default="auto", choices=["auto", "0", "1", "comm"],
                    help="with --simulate-world: the captured step's exchange placement "
                         "(parallel/engine.py set_graph_overlap)")
    ap.add_argument("--sim-all", action="store_true",
                    help="with --simulate-world: the ResNet-50 BASELINE configs (layer-wise "
                         "Top-K 0.1 %%, entire-model QSGD 8-bit) instead of the given method")
    ap.add_argument("--graph", default="on", choices=["on", "off"],
                    help="on: after 3 eager warm-up steps capture the whole step (fwd, bwd, "
                         "per-bucket compression + collectives + decode/SGD inline in backward "
                         "order) as one HIP graph and replay it (train/imagenet.py "
                         "ImageNetTrainer)")
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


def _reference_key(args) -> str:
    """accuracy_reference.json's name for this run's method ('' when it has none)."""
    if args.compress == "none" or args.method == "none":
        return "none"
    if args.compress != "layerwise" or args.method != "Topk" or args.ratio != 0.001:
        return ""
    return ("topk0.1%" + ("+ef" if args.ef else "") + ("+mc" if args.momentum_correction else "")
            + ("+dense4k" if args.ef_dense_below == 4096 else ""))


def _reference_mean(steps: int, key: str):
    """(3-seed mean, per-seed top-1) of ``key`` at this step budget from accuracy_reference.json,
    or (None, None)."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "layer_wise_aaai20_amd",
                        "train", "accuracy_reference.json")
    try:
        with open(path) as f:
            ref = json.load(f)
    except (OSError, ValueError):
        return None, None
    v = ref.get("methods", {}).get(key) if int(ref.get("steps", -1)) == int(steps) else None
    return (v["mean"], v["top1"]) if v else (None, None)


def _reference_points(steps: int) -> str:
    """Reference points for the printed top-1, measured at the same step budget over several
    seeds (layer_wise_aaai20_amd/train/accuracy_reference.json, folded by scripts/acc_reference.py
    from scripts/accuracy_r50.py runs; the raw runs are in profiles/r4/)."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "layer_wise_aaai20_amd",
                        "train", "accuracy_reference.json")
    try:
        with open(path) as f:
            ref = json.load(f)
    except (OSError, ValueError):
        return ""
    if int(ref.get("steps", -1)) != int(steps):
        return ""
    parts = [f"{k}: {v['mean']:.1f}% (seeds {', '.join(f'{x:.1f}' for x in v['top1'])})"
             for k, v in ref.get("methods", {}).items()]
    return ("; reference points at this budget (bf16, 3 seeds), " + "; ".join(parts) +
            " (layer_wise_aaai20_amd/train/accuracy_reference.json)")


def simulate(args) -> None:
    """--simulate-world W (train/simworld.py): JSON lines, no benchmark line."""
    from layer_wise_aaai20_amd.train.simworld import simulate_imagenet
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if args.sim_all:
        cfgs = [dict(compress="layerwise", method="Topk", K=0.001),
                dict(compress="entiremodel", method="RandomDithering", qstates=255)]
    else:
        cfgs = [dict(compress=args.compress, method=args.method, K=args.ratio,
                     qstates=args.qstates, error_feedback=args.ef,
                     dense_below=args.ef_dense_below,
                     momentum_correction=args.momentum_correction)]
    for c in cfgs:
        line = simulate_imagenet(args.simulate_world, dev, steps=args.steps,
                                 warmup=max(3, args.warmup), model=args.model,
                                 batch=args.batch, image_size=args.image_size, dtype=args.dtype,
                                 bucket_mb=args.bucket_mb, sim_wire=args.sim_wire,
                                 overlap=args.sim_overlap, **c)
        line["data"] = "synthetic (random uint8 images, random-init weights)"
        print(json.dumps(line), flush=True)
        if args.json_out:
            with open(args.json_out, "a") as f:
                f.write(json.dumps(line) + "\n")


def main():
    args = parse()
    if args.simulate_world > 1:
        simulate(args)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    if args.share_gpu:
        local = 0
        if world > 1 and args.backend == "nccl":
            # RCCL refuses two ranks on one device of one host; distinct host ids make it treat
            # them as separate nodes (socket transport) — set before anything touches RCCL
            os.environ["NCCL_HOSTID"] = f"lwaaai-rank{rank}"
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
                       dense_below=args.ef_dense_below,
                       momentum_correction=args.momentum_correction, fused=not args.no_fused, momentum=0.9, weight_decay=1e-4, no_bn_wd=True,
                       lr=0.1, graph=args.graph == "on" and args.warmup >= 2,
                       # capture inside the untimed warm-up: at least one eager step (tile tuner,
                       # lazily built device tables, allocator, RCCL warm), then capture + replay
                       graph_warmup=max(1, min(3, args.warmup - 1)),
                       # no graph-vs-eager timing decision: it would spill syncs into the timed
                       # steps (the captured ResNet-50 step is the faster one: 24.3 vs 27.2 ms)
                       graph_auto=False)
    B, S = args.batch, args.image_size
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    # class-conditional synthetic images (a per-class colour offset on uniform noise): a short
    # run can learn the signal, so the held-out top-1 printed below means something. A pool of
    # batches, generated before timing, is cycled through the steps.
    bias = torch.randint(0, 128, (1000, 3), dtype=torch.int16, device=dev,
                         generator=torch.Generator(device=dev).manual_seed(7))

    def make_batch(gen):
        t = torch.randint(0, 1000, (B,), device=dev, generator=gen)
        x = torch.randint(0, 128, (B, S, S, 3), dtype=torch.int16, device=dev, generator=gen)
        return (x + bias[t].view(B, 1, 1, 3)).to(torch.uint8), t
    pool = [make_batch(g) for _ in range(args.pool)]

    beat = _Heartbeat(rank)
    for i in range(args.warmup):
        tr.step(*pool[i % len(pool)])
        beat.note(f"warmup {i + 1}/{args.warmup}")
    beat.stop()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        tr.step(*pool[(args.warmup + i) % len(pool)])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms = dt / args.steps * 1e3
    graphed = tr.graph_replays >= args.steps
    # ---- outside the timed region: per-bucket compress / exchange / decode µs of one step,
    # then the accuracy half of the metric (a short training run of the same configuration)
    eng = tr.ddp.engine
    eng.timing = True
    tr.step(*pool[0])
    bucket_us = eng.read_timings()
    eng.timing = False
    stats = tr.ddp.sync_stats()
    overflow = eng.read_overflow()
    acc = None
    if args.acc_steps > 0:
        del tr                            # (free the 224 px trainer's graph pool first)
        torch.cuda.empty_cache()
        from layer_wise_aaai20_amd.train.accuracy import short_run_top1
        acc = short_run_top1(dev, steps=args.acc_steps, size=128, batch=256, rank=rank,
                             world=world, compress=args.compress, method=args.method,
                             K=args.ratio, V=args.threshold, qstates=args.qstates,
                             error_feedback=args.ef, dtype=args.dtype,
                             dense_below=args.ef_dense_below,
                             momentum_correction=args.momentum_correction)
    value = world * B * args.steps / dt
    default = (args.model == "resnet50" and args.compress == "layerwise" and args.method == "Topk"
               and args.ratio == 0.001 and not args.ef and args.ef_dense_below == 0
               and not args.momentum_correction)
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
        "data": "synthetic (class-conditional random uint8 224x224 images, pool of 4 batches; "
                "random-init weights)",
        "top1": acc["top1"] if acc else None,
        # the same method's 3-seed mean at this budget (this run is seed 0 of it)
        "top1_3seed_mean": (_reference_mean(acc["steps"], _reference_key(args))[0]
                            if acc else None),
        "top1_3seed": (_reference_mean(acc["steps"], _reference_key(args))[1]
                       if acc else None),
        "top1_note": (f"held-out top-1 (%) of a fresh ResNet-50 trained {acc['steps']} steps with "
                      f"the same compression at {acc['image_size']} px, {acc['per_gpu_batch']}/GPU "
                      f"(linear LR warm-up to 1.0 at batch 512, linear decay to 0, graph step, "
                      f"kernel choices pinned by the shipped "
                      f"gfx950 tuning table) on the class-conditional synthetic task; "
                      f"chance 0.1%; top-5 {acc['top5']}%; train loss {acc['loss_first20']} -> "
                      f"{acc['loss_last20']} (train/accuracy.py)" + _reference_points(acc['steps'])
                      if acc else "not measured (--acc-steps 0)"),
        "hip_graph": graphed,
        "comm": {"backend": dist.get_backend() if world > 1 else "none (1 rank)",
                 "world_size": dist.get_world_size() if world > 1 else 1,
                 "bucket_us": [{k: (round(v, 1) if isinstance(v, float) else v)
                                for k, v in b.items()} for b in bucket_us]},
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
            "ef_dense_below": args.ef_dense_below,
            "momentum_correction": args.momentum_correction,
            "wire_bytes_per_rank": stats.payload_bytes,
            "selection_overflow": overflow,
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
        # the result line is out: a teardown that blocks must not turn a finished run into a
        # hung one. faulthandler's watchdog is a C thread (it needs no GIL, which a blocked
        # native call may hold): it ends the process if the clean teardown takes over a minute
        import faulthandler
        sys.stdout.flush()
        faulthandler.dump_traceback_later(60, exit=True)
        from layer_wise_aaai20_amd.parallel import comm as _comm
        _comm.shutdown_native()           # captured graphs released, then local aborts
        dist.destroy_process_group()
        faulthandler.cancel_dump_traceback_later()


if __name__ == "__main__":
    main()
