"""A world of W ranks timed on ONE GPU (``bench.py --simulate-world W``,
``bench_cifar.py --simulate-world W``).

The driver's 8-GPU scaling run is the measurement that counts; this is the cost model that can be
run on the 1-GPU boxes before it. The trainer is built for W ranks (codecs, payload sizes, the
W-rank decode, the side-stream compression branch inside the captured step graph that world > 1
uses) and its communicator is the loopback one (``parallel/loopback.py``) in frozen mode: the W-1
peers' payloads are compressed once and then replayed, so a step costs this GPU what it costs a
real rank — its own compression, the W·payload bytes landing in memory, the decode of every
rank's contribution — and not the peers' compressions, which a real node runs on the other GPUs.

Reported per configuration (one JSON line):

* ``ms_per_step`` — the simulated world-W step (HIP graph replay);
* ``ms_compute_only`` — the same model and batch with no compression and no exchange (world 1,
  method none): forward, backward and SGD only; both timed in alternating windows (3 rounds,
  medians) in one process;
* ``exposed_ms`` / ``exposed_pct`` — their difference, as a share of the simulated step: the
  compression / decode work not hidden behind backward plus the exchange. With ``wire=True``
  (``bench.py --sim-wire``) every collective also pays its modelled xGMI transfer time as a busy
  kernel on ``cus`` workgroups (``parallel/loopback.py WireModel``: ``link_gbs`` GB/s per xGMI
  link, one link per peer — MI355X: 7 links per GPU, full mesh — all-gather = payload / link,
  all-reduce = 2 · bytes / (W · link), grouped send/recv = largest message / link, plus
  ``latency_us`` each), so the exposure includes the wire wherever the step's schedule leaves it
  exposed; ``overlap`` picks the captured step's exchange placement (engine
  ``set_graph_overlap``). Without the wire, ``xgmi_model_ms`` prices the last bucket's exchange
  separately;
* per-bucket ``compress_us`` / ``decode_us`` of one eager step (HIP events on the side stream).

Reference the mechanism replaces: ``CIFAR10/core.py:227-301`` (entire-model exchange),
``IMAGENET/training/sparsified_ddp.py:403-452`` (overlap with backward)."""
from __future__ import annotations

import time
from typing import Callable, Dict, List

import torch

LINK_GBS = 100.0          # effective xGMI GB/s per link and direction assumed by the model
LATENCY_US = 15.0         # per collective
WIRE_CUS = 16             # workgroups a simulated transfer keeps busy (RCCL channels)


def _time(step: Callable[[], None], warmup: int, steps: int) -> float:
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def _alternate(step_a: Callable[[], None], step_b: Callable[[], None], warmup: int, steps: int,
               rounds: int = 3):
    """Median ms/step of two steps timed in alternating windows (A B A B ...): the difference of
    two configurations is then measured under the same clock / thermal state, which one-shot
    windows on different boxes were not (the same simulated AlexNet step read 0.845 and
    0.866 ms)."""
    import statistics
    ta, tb = [], []
    for r in range(rounds):
        ta.append(_time(step_a, warmup if r == 0 else 2, steps))
        tb.append(_time(step_b, warmup if r == 0 else 2, steps))
    return statistics.median(ta), statistics.median(tb)


def _frozen_peers(engine, world: int, seed: int = 0, scale: float = 1e-3, wire: bool = False,
                  overlap: str = "auto"):
    from ..parallel.loopback import WireModel, attach_loopback
    g = torch.Generator(device=engine.device).manual_seed(seed)
    peers = [torch.randn(engine.arena.numel, device=engine.device, generator=g) * scale
             for _ in range(world - 1)]
    wm = WireModel(LINK_GBS, LATENCY_US, WIRE_CUS) if wire else None
    lb = attach_loopback(engine, peers, frozen=True, wire_model=wm)
    engine.set_graph_overlap(overlap)
    return lb


def _wire_fields(lb, engine, overlap: str) -> Dict:
    wm = lb.wire_model
    out = {"overlap_mode": engine.graph_overlap_mode(), "overlap_requested": overlap,
           "wire_priced": wm is not None}
    if wm is not None:
        out["wire_model"] = {"gbs_per_link": wm.link_gbs, "latency_us": wm.latency_us,
                             "cus": wm.cus}
    return out


def xgmi_model_ms(codec, payload_bytes: int, world: int, link_gbs: float = LINK_GBS,
                  latency_us: float = LATENCY_US) -> float:
    """Wire time of one bucket's collective on a W-GPU full xGMI mesh (see module doc)."""
    if world <= 1:
        return 0.0
    if codec.collective == "all_gather":
        t = payload_bytes / (link_gbs * 1e9)
    elif codec.collective == "quant_rs":            # two grouped send/recv phases of ~1/W each
        t = payload_bytes / ((world - 1) * link_gbs * 1e9)
    else:
        t = 2.0 * payload_bytes / (world * link_gbs * 1e9)
    return (t + latency_us * 1e-6) * 1e3


def _engine_report(engine, world: int, bucket_us: List[dict]) -> Dict:
    last = len(engine.buckets) - 1
    codec = engine.codecs[last]
    # the last bucket's payload (the one exchanged after backward)
    pay = int(getattr(codec, "last_payload_bytes", 0))
    return {"buckets": len(engine.buckets),
            "codecs": sorted({c.name for c in engine.codecs}),
            "wire_bytes_per_rank": int(engine.stats.payload_bytes),
            "recv_bytes_per_rank": int(sum(
                (world - 1) * c.last_payload_bytes if c.collective == "all_gather" else
                c.last_payload_bytes if c.collective == "quant_rs" else
                2 * (world - 1) * c.last_payload_bytes // world for c in engine.codecs)),
            "last_bucket_payload_bytes": pay,
            "xgmi_model_ms_last_bucket": round(xgmi_model_ms(codec, pay, world), 4),
            "xgmi_model_ms_all_buckets": round(sum(
                xgmi_model_ms(c, int(c.last_payload_bytes), world) for c in engine.codecs), 4),
            "bucket_us": [{k: (round(v, 1) if isinstance(v, float) else v) for k, v in b.items()}
                          for b in bucket_us]}


def simulate_imagenet(world: int, device, steps: int = 10, warmup: int = 6, model="resnet50",
                      compress="layerwise", method="Topk", K=0.001, qstates=255,
                      error_feedback=False, batch=256, image_size=224, dtype="bf16",
                      bucket_mb=50.0, wire="auto", dense_below=0,
                      momentum_correction=False, sim_wire: bool = False,
                      overlap: str = "auto") -> Dict:
    from .imagenet import build_trainer
    dev = torch.device(device)
    g = torch.Generator(device=dev).manual_seed(1234)
    x = torch.randint(0, 256, (batch, image_size, image_size, 3), dtype=torch.uint8, device=dev,
                      generator=g)
    t = torch.randint(0, 1000, (batch,), device=dev, generator=g)
    common = dict(model=model, device=dev, dtype=dtype, bucket_cap_mb=bucket_mb, lr=0.1,
                  graph=True, graph_warmup=2, graph_auto=False)
    base = build_trainer(compress="none", method="none", world_size=1, **common)
    tr = build_trainer(compress=compress, method=method, K=K, qstates=qstates,
                       error_feedback=error_feedback, wire=wire, world_size=world,
                       dense_below=dense_below, momentum_correction=momentum_correction,
                       **common)
    eng = tr.ddp.engine
    lb = _frozen_peers(eng, world, wire=sim_wire, overlap=overlap)
    t_base, t_sim = _alternate(lambda: base.step(x, t), lambda: tr.step(x, t), warmup, steps)
    del base
    torch.cuda.empty_cache()
    replays = tr.graph_replays
    eng.timing = True
    tr.step(x, t)
    bucket_us = eng.read_timings()
    eng.timing = False
    out = {"config": f"{model} {compress} {method}" +
                     (f" K={K}" if method in ("Topk", "Randomk") else "") +
                     (f" Q={qstates}" if method == "RandomDithering" else "") +
                     (" +EF" if error_feedback else ""),
           "world_sim": world, "per_gpu_batch": batch, "image_size": image_size, "dtype": dtype,
           "ms_per_step": round(t_sim, 3), "ms_compute_only": round(t_base, 3),
           "exposed_ms": round(t_sim - t_base, 3),
           "exposed_pct": round(100.0 * (t_sim - t_base) / t_sim, 2),
           "img_per_s_per_gpu": round(batch / t_sim * 1e3, 1),
           "hip_graph": replays >= steps, "wire": wire,
           "link_model": {"gbs_per_link": LINK_GBS, "latency_us": LATENCY_US}}
    out.update(_wire_fields(lb, eng, overlap))
    out.update(_engine_report(eng, world, bucket_us))
    del tr
    torch.cuda.empty_cache()
    return out


def simulate_cifar(world: int, device, name: str, cfg: Dict, steps: int = 30,
                   warmup: int = 8, sim_wire: bool = False, overlap: str = "auto") -> Dict:
    from .cifar_fast import CifarTrainer
    dev = torch.device(device)
    base = CifarTrainer(device=dev, n_train=512 * 12, graph=True, network=cfg["network"],
                        compress="none", method="none")
    base.graphed.warmup = 2
    tr = CifarTrainer(device=dev, n_train=512 * 12, graph=True, world_size=world, **cfg)
    tr.graphed.warmup = 2
    eng = tr.ddp.engine
    lb = _frozen_peers(eng, world, wire=sim_wire, overlap=overlap)
    t_base, t_sim = _alternate(lambda: base.step(), lambda: tr.step(), warmup, steps)
    del base
    torch.cuda.empty_cache()
    replays = tr.graphed.replays
    eng.timing = True
    tr.step()
    bucket_us = eng.read_timings()
    eng.timing = False
    out = {"config": f"cifar {name}: {cfg['network']} {cfg['compress']} {cfg['method']}" +
                     (f" K={cfg['K']}" if "K" in cfg else "") +
                     (" +EF" if cfg.get("error_feedback") else ""),
           "world_sim": world, "per_gpu_batch": tr.bs,
           "ms_per_step": round(t_sim, 3), "ms_compute_only": round(t_base, 3),
           "exposed_ms": round(t_sim - t_base, 3),
           "exposed_pct": round(100.0 * (t_sim - t_base) / t_sim, 2),
           "img_per_s_per_gpu": round(tr.bs / t_sim * 1e3, 1),
           "hip_graph": replays >= steps,
           "link_model": {"gbs_per_link": LINK_GBS, "latency_us": LATENCY_US}}
    out.update(_wire_fields(lb, eng, overlap))
    out.update(_engine_report(eng, world, bucket_us))
    return out
