"""Timers, loggers and meters (SURVEY.md §5 "Metrics / logging / observability").

CIFAR side (``CIFAR10/core.py:14-37, 157-173``, ``dawn.py:89-96``): ``Timer``, ``TableLogger``,
``TSVLogger``, ``StatsLogger``, ``PiecewiseLinear``. ImageNet side
(``IMAGENET/training/meter.py``, ``logger.py``): ``AverageMeter``, ``TimeMeter``, ``NetworkMeter``,
``TensorboardLogger`` (tensorboardX / wandb when importable, otherwise a JSONL event file),
``FileLogger`` (``verbose.log`` / ``event.log`` / ``debug.log``, master only). New: ``CommMeter``
with compression statistics (density, bytes on the wire, compress / comm µs).
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time
from collections import namedtuple
from typing import Callable, Dict, Iterable, Optional

import numpy as np
import torch


# ------------------------------------------------------------------------------ CIFAR side
class Timer:
    """Lap timer; ``synch`` (e.g. ``torch.cuda.synchronize``) is called before every reading."""

    def __init__(self, synch: Optional[Callable] = None):
        self.synch = synch or (lambda: None)
        self.synch()
        self.times = [time.time()]
        self.total_time = 0.0

    def __call__(self, include_in_total: bool = True) -> float:
        self.synch()
        self.times.append(time.time())
        dt = self.times[-1] - self.times[-2]
        if include_in_total:
            self.total_time += dt
        return dt


def localtime() -> str:
    return time.strftime("%Y-%m-%d %H:%M:%S", time.localtime())


class TableLogger:
    def __init__(self, file=None):
        self.file = file or sys.stdout

    def append(self, output: dict) -> None:
        if not hasattr(self, "keys"):
            self.keys = list(output.keys())
            print(*(f"{k:>12s}" for k in self.keys), file=self.file)
        vals = [output[k] for k in self.keys]
        print(*(f"{v:12.4f}" if isinstance(v, (float, np.floating)) else f"{v:12}" for v in vals),
              file=self.file)


class TSVLogger:
    """``logs.tsv`` writer: ``epoch\\thours\\ttop1Accuracy`` (``dawn.py:89-96``)."""

    def __init__(self):
        self.log = ["epoch\thours\ttop1Accuracy"]

    def append(self, output: dict) -> None:
        epoch, hours, acc = output["epoch"], output["total time"] / 3600, output["test acc"] * 100
        self.log.append(f"{epoch}\t{hours:.8f}\t{acc:.2f}")

    def __str__(self) -> str:
        return "\n".join(self.log)


class PiecewiseLinear(namedtuple("PiecewiseLinear", ("knots", "vals"))):
    def __call__(self, t):
        return float(np.interp([t], self.knots, self.vals)[0])


class StatsLogger:
    """Keeps per-batch stats on device; one host sync per epoch (``core.py:161-173``)."""

    def __init__(self, keys=("loss", "correct")):
        self._stats = {k: [] for k in keys}

    def append(self, output: dict) -> None:
        for k, v in self._stats.items():
            v.append(output[k].detach())

    def stats(self, key) -> torch.Tensor:
        return torch.cat([t.reshape(-1) for t in self._stats[key]])

    def mean(self, key) -> float:
        t = self.stats(key)
        return float(t.float().mean().item()) if t.numel() else float("nan")


# ------------------------------------------------------------------------------ ImageNet side
class AverageMeter:
    def __init__(self):
        self.reset()

    def reset(self):
        self.val = self.avg = self.sum = 0.0
        self.count = 0

    def update(self, val, n=1):
        self.val = float(val)
        self.sum += float(val) * n
        self.count += n
        self.avg = self.sum / max(self.count, 1)


class TimeMeter:
    """Batch time vs data-loading time (``meter.py:49-60``)."""

    def __init__(self):
        self.batch_time = AverageMeter()
        self.data_time = AverageMeter()
        self.start = time.time()

    def batch_start(self):
        self.data_time.update(time.time() - self.start)

    def batch_end(self):
        self.batch_time.update(time.time() - self.start)
        self.start = time.time()


def network_bytes():
    """Host NIC rx/tx byte counters from ``/proc/net/dev`` (``meter.py:66-86``)."""
    try:
        with open("/proc/net/dev") as f:
            lines = f.readlines()[2:]
    except OSError:
        return 0, 0
    rx = tx = 0
    for ln in lines:
        name, data = ln.split(":", 1)
        if name.strip() == "lo":
            continue
        f = data.split()
        rx += int(f[0])
        tx += int(f[8])
    return rx, tx


class NetworkMeter:
    def __init__(self):
        self.recv, self.sent = network_bytes()
        self.t = time.time()

    def update_bandwidth(self):
        rx, tx = network_bytes()
        now = time.time()
        dt = max(now - self.t, 1e-9)
        recv_gbit = (rx - self.recv) * 8 / dt / 1e9
        sent_gbit = (tx - self.sent) * 8 / dt / 1e9
        self.recv, self.sent, self.t = rx, tx, now
        return recv_gbit, sent_gbit


class CommMeter:
    """Compression statistics from a GradSyncEngine (new)."""

    def __init__(self, engine):
        self.engine = engine

    def snapshot(self) -> Dict[str, float]:
        st = self.engine.stats
        return {"comm/payload_bytes": st.payload_bytes, "comm/dense_bytes": st.dense_bytes,
                "comm/ratio": st.ratio, "comm/buckets": st.buckets}


class NoOp:
    def __getattr__(self, *args):
        def no_op(*a, **k):
            pass
        return no_op


class TensorboardLogger:
    """Scalars with step = cumulative examples (``logger.py:13-68``). Writes via tensorboardX or
    wandb when importable; always mirrors to ``<logdir>/scalars.jsonl``."""

    def __init__(self, output_dir: str = "", is_master: bool = True):
        self.is_master = is_master and bool(output_dir)
        self.step = 0
        self.current_time = time.time()
        self.writer = None
        self.jsonl = None
        if self.is_master:
            os.makedirs(output_dir, exist_ok=True)
            self.jsonl = open(os.path.join(output_dir, "scalars.jsonl"), "a")
            try:
                from tensorboardX import SummaryWriter  # optional
                self.writer = SummaryWriter(output_dir)
            except Exception:
                self.writer = None

    def log(self, tag, val):
        if not self.is_master:
            return
        v = float(val)
        if self.writer is not None:
            self.writer.add_scalar(tag, v, self.step)
        self.jsonl.write(json.dumps({"step": self.step, "tag": tag, "value": v}) + "\n")

    def update_step_count(self, batch_total):
        self.step += batch_total

    def log_memory(self):
        if torch.cuda.is_available():
            self.log("memory/allocated_gb", torch.cuda.memory_allocated() / 1e9)
            self.log("memory/max_allocated_gb", torch.cuda.max_memory_allocated() / 1e9)
            self.log("memory/cached_gb", torch.cuda.memory_reserved() / 1e9)

    def log_trn_times(self, batch_time, data_time, batch_size):
        self.log("times/step", 1000 * batch_time)
        self.log("times/data", 1000 * data_time)
        images_per_sec = batch_size / max(batch_time, 1e-9)
        self.log("times/1gpu_images_per_sec", images_per_sec)
        self.log("times/8gpu_images_per_sec", 8 * images_per_sec)

    def log_size(self, bs=None, sz=None):
        if bs:
            self.log("sizes/batch", bs)
        if sz:
            self.log("sizes/image", sz)

    def log_trn_loss(self, loss, top1, top5):
        self.log("losses/xent", loss)          # reference tags (logger.py:50-53)
        self.log("losses/train_1", top1)
        self.log("losses/train_5", top5)

    def log_comm(self, stats, bucket_us=None):
        """Compression telemetry (SURVEY.md §5 metrics row): bytes this rank put on the wire last
        step, their ratio to the dense fp32 gradient, and per-bucket compress / exchange / decode
        µs when the engine timed the step."""
        self.log("comm/payload_bytes", stats.payload_bytes)
        self.log("comm/dense_bytes", stats.dense_bytes)
        self.log("comm/ratio", stats.ratio)
        self.log("comm/overflow", getattr(stats, "overflow", 0))
        for b in bucket_us or []:
            i = b["bucket"]
            for k in ("compress_us", "exchange_us", "idle_us", "decode_us"):
                if b.get(k) is not None:
                    self.log(f"comm/bucket{i}_{k}", b[k])

    def log_eval(self, top1, top5, time_):
        self.log("losses/test_1", top1)
        self.log("losses/test_5", top5)
        self.log("times/eval_sec", time_)

    def close(self):
        if self.writer is not None:
            self.writer.close()
        if self.jsonl is not None:
            self.jsonl.close()


class FileLogger:
    """``verbose.log`` / ``event.log`` / ``debug.log`` in ``output_dir``, master only
    (``logger.py:74-121``)."""

    def __init__(self, output_dir: str = "", is_master: bool = True, is_rank0: bool = True):
        self.output_dir = output_dir
        self.is_master = is_master
        self.is_rank0 = is_rank0
        if not is_rank0:
            self.logger = NoOp()
            return
        self.logger = logging.getLogger(f"lwaaai.{id(self)}")
        self.logger.setLevel(logging.DEBUG)
        self.logger.propagate = False
        fmt = logging.Formatter("%(message)s")
        ch = logging.StreamHandler(sys.stdout)
        ch.setLevel(logging.DEBUG)
        ch.setFormatter(fmt)
        self.logger.addHandler(ch)
        if output_dir and is_master:
            os.makedirs(output_dir, exist_ok=True)
            for name, lvl in (("debug.log", logging.DEBUG), ("verbose.log", logging.INFO),
                              ("event.log", logging.WARNING)):
                fh = logging.FileHandler(os.path.join(output_dir, name))
                fh.setLevel(lvl)
                fh.setFormatter(fmt)
                self.logger.addHandler(fh)

    def console(self, *args):
        self.logger.debug(*args)

    def event(self, *args):
        self.logger.warning(*args)

    def verbose(self, *args):
        self.logger.info(*args)
