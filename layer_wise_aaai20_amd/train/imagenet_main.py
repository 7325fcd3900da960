"""ImageNet ResNet training entry point with the reference CLI
(``IMAGENET/training/train_imagenet_nv.py:39-253, 388-651``).

    torchrun --nproc-per-node 8 -m IMAGENET.training.train_imagenet_nv /data/imagenet \
        --logdir runs/x --distributed --init-bn0 --no-bn-wd -c layerwise --method Topk -K 0.001

Kept: every reference flag, the progressive-resizing phase schedule (honoured from ``--phases``,
D14), LR warm-up ``Scheduler``, ``DataManager`` phase swaps, per-step cross-rank metric reduction,
sharded distributed evaluation with uneven batches (``distributed_predict``), ``event.log`` /
TensorBoard tags, checkpoint layout ``{epoch, state_dict, best_top5, optimizer}``, ``--resume``.

Fixed: duplicate ``--momentum`` (D4, one flag, default 0.9), ``world_size`` is the
process-group size (D5), ``enitremodel`` really runs entire-model compression (D3), no double
reduction after ``--ddp`` / ``--sparsification`` (D11), fp32 ``--no-bn-wd`` keeps every parameter
(D12), loader dtype follows the model (D13).

Added: ``--bf16`` (autocast, the MI355X default), ``--overlap`` (CompressedDDP: compression of each
bucket overlapped with backward), ``--error-feedback``, ``--wire``, ``--arch``, ``--epochs``,
``--synthetic-size``, ``--extra-ckpt`` (also saves EF residuals / scheduler state).
"""
from __future__ import annotations

import argparse
import ast
import copy
import json
import os
import shutil
import sys
import time
from datetime import datetime

import torch
import torch.distributed as dist
from torch import nn

from ..data import imagenet as D
from ..models import resnet as R
from ..ops import nn as lwnn
from ..ops._ext import h16, set_half
from ..parallel import comm
from ..parallel import functional as F
from ..parallel.ddp import CompressedDDP, DistributedDataParallel, RandomKSparsifiedDDP
from ..utils import fp16 as fp16util
from ..utils.logging import AverageMeter, FileLogger, NetworkMeter, TensorboardLogger, TimeMeter

from .graphs import StepGraph
from .schedules import NAMES as _SCHED_NAMES, schedule as _schedule


def get_parser():
    p = argparse.ArgumentParser(description="ImageNet training with compressed gradients")
    p.add_argument("data", metavar="DIR", nargs="?", default="synthetic", help="dataset path")
    p.add_argument("--phases", type=str, default="one_machine",
                   help="schedule name, or a JSON / python-literal list of phase dicts")
    p.add_argument("-j", "--workers", default=0, type=int)
    p.add_argument("--start-epoch", default=0, type=int)
    p.add_argument("--momentum", default=0.9, type=float)
    p.add_argument("--weight-decay", "--wd", default=1e-4, type=float)
    p.add_argument("--init-bn0", action="store_true")
    p.add_argument("--print-freq", "-p", default=50, type=int)
    p.add_argument("--no-bn-wd", action="store_true")
    p.add_argument("--resume", default="", type=str)
    p.add_argument("-e", "--evaluate", dest="evaluate", action="store_true")
    p.add_argument("--fp16", action="store_true")
    p.add_argument("--bf16", action="store_true")
    p.add_argument("--no-graph", action="store_true",
                   help="fused path: launch every kernel from Python instead of replaying the "
                        "captured HIP graph of the step")
    p.add_argument("--loss-scale", type=float, default=1024)
    p.add_argument("--distributed", action="store_true")
    p.add_argument("--dist-url", default="env://", type=str)
    p.add_argument("--dist-backend", default=None, type=str)
    p.add_argument("--local_rank", "--local-rank", default=None, type=int)
    p.add_argument("--logdir", default="", type=str)
    p.add_argument("--name", type=str, default="imagenet")
    p.add_argument("--short-epoch", action="store_true")
    p.add_argument("--log_all_workers", type=int, default=0)
    p.add_argument("--sparsification", action="store_true")
    p.add_argument("--randk", type=float, default=1)
    p.add_argument("--ddp", action="store_true")
    p.add_argument("--seed", type=int, default=2147483647)
    p.add_argument("--compress", "-c", type=str, default="none")
    p.add_argument("--method", type=str, default="none")
    p.add_argument("--ratio", "-K", type=float, default=0.5)
    p.add_argument("--threshold", "-V", type=float, default=0.001)
    p.add_argument("--qstates", "-Q", type=int, default=255)
    # additions
    p.add_argument("--arch", default="resnet50")
    p.add_argument("--overlap", action="store_true", help="CompressedDDP (bucketed, overlapped)")
    p.add_argument("--error-feedback", action="store_true")
    # opt-in EF variants (fused path; profiles/r4/ef_root_cause.md)
    p.add_argument("--ef-dense-below", type=int, default=0,
                   help="send tensors of at most this many elements densely (e.g. 4096: BN "
                        "parameters and biases)")
    p.add_argument("--momentum-correction", action="store_true",
                   help="DGC momentum correction: the velocity lives in the EF residual and the "
                        "optimizer runs without momentum")
    p.add_argument("--wire", default="auto", choices=["auto", "sparse", "sparse-exact", "sparse-capped", "dense", "indexfree", "qrs"])
    p.add_argument("--epochs", type=int, default=None, help="stop after this many epochs")
    p.add_argument("--synthetic-size", type=int, default=None,
                   help="synthetic train images per phase (default 64 batches)")
    p.add_argument("--no-fused", action="store_true",
                   help="torch convs / BN, post-backward sync, torch SGD (the reference's path)")
    p.add_argument("--extra-ckpt", action="store_true")
    p.add_argument("--device", default=None)
    return p


def parse_phases(spec: str):
    if spec in _SCHED_NAMES or spec == "smoke":
        return _schedule(spec)
    if spec.isdigit():
        return _schedule(int(spec))
    try:
        return json.loads(spec)
    except json.JSONDecodeError:
        return ast.literal_eval(spec)


def adapt_state_dict(sd: dict, model) -> dict:
    """Checkpoints written under a DP wrapper carry a ``module.`` key prefix
    (``train_imagenet_nv.py:663-669``); add or strip it so a checkpoint loads into a wrapped or a
    bare model alike (e.g. ``--evaluate`` without ``--distributed``)."""
    want = next(iter(model.state_dict()), "")
    have = next(iter(sd), "")
    if want.startswith("module.") and not have.startswith("module."):
        return {"module." + k: v for k, v in sd.items()}
    if have.startswith("module.") and not want.startswith("module."):
        return {k[len("module."):]: v for k, v in sd.items()}
    return sd


def listify(p=None, q=None):
    """``listify`` of train_imagenet_nv.py:691-699 without ``collections.Iterable`` (D9)."""
    if p is None:
        p = []
    elif not isinstance(p, (list, tuple)):
        p = [p]
    p = list(p)
    n = q if isinstance(q, int) else 1 if q is None else len(q)
    if len(p) == 1:
        p = p * n
    return p


def to_python_float(t):
    if isinstance(t, (float, int)):
        return t
    return t.item() if hasattr(t, "item") else t[0]


def correct(output, target, topk=(1,)):
    maxk = min(max(topk), output.size(1))
    _, pred = output.topk(maxk, 1, True, True)
    pred = pred.t()
    ok = pred.eq(target.view(1, -1).expand_as(pred))
    return [ok[:min(k, maxk)].reshape(-1).float().sum(0, keepdim=True) for k in topk]


def accuracy(output, target, topk=(1,)):
    bs = target.size(0)
    return [c.mul_(100.0 / bs) for c in correct(output, target, topk)]


# ------------------------------------------------------------------------------------ scheduler
class Scheduler:
    """Per-iteration piecewise-constant / linear LR from the phase list (train_imagenet_nv.py:602)."""

    def __init__(self, optimizer, phases, log=None, tb=None, momentum=None):
        self.optimizer = optimizer
        self.current_lr = None
        self.phases = [self.format_phase(p) for p in phases]
        self.tot_epochs = max(max(p["ep"]) for p in self.phases)
        self.log, self.tb, self.momentum = log, tb, momentum

    @staticmethod
    def format_phase(phase):
        phase["ep"] = listify(phase["ep"])
        phase["lr"] = listify(phase["lr"])
        if len(phase["lr"]) == 2:
            assert len(phase["ep"]) == 2, "Linear learning rates must contain end epoch"
        return phase

    @staticmethod
    def calc_linear_lr(lr_start, lr_end, epoch_curr, batch_curr, epoch_tot, batch_tot):
        step_tot = epoch_tot * batch_tot
        step_curr = epoch_curr * batch_tot + batch_curr
        return lr_start + step_curr * (lr_end - lr_start) / step_tot

    def linear_phase_lr(self, phase, epoch, batch_curr, batch_tot):
        lr_start, lr_end = phase["lr"]
        ep_start, ep_end = phase["ep"]
        if "epoch_step" in phase:
            batch_curr = 0
        return self.calc_linear_lr(lr_start, lr_end, epoch - ep_start, batch_curr,
                                   ep_end - ep_start, batch_tot)

    def get_current_phase(self, epoch):
        for phase in reversed(self.phases):
            if epoch >= phase["ep"][0]:
                return phase
        raise Exception("Epoch out of range")

    def get_lr(self, epoch, batch_curr, batch_tot):
        phase = self.get_current_phase(epoch)
        if len(phase["lr"]) == 1:
            return phase["lr"][0]
        return self.linear_phase_lr(phase, epoch, batch_curr, batch_tot)

    def update_lr(self, epoch, batch_num, batch_tot):
        lr = self.get_lr(epoch, batch_num, batch_tot)
        if self.current_lr == lr:
            return
        if self.log and (batch_num == 1 or batch_num == batch_tot):
            self.log.event(f"Changing LR from {self.current_lr} to {lr}")
        self.current_lr = lr
        for g in self.optimizer.param_groups:
            g["lr"] = lr
        if self.tb:
            self.tb.log("sizes/lr", lr)
            self.tb.log("sizes/momentum", self.momentum)

    def state_dict(self):
        return {"current_lr": self.current_lr}

    def load_state_dict(self, sd):
        self.current_lr = sd.get("current_lr")


# ------------------------------------------------------------------------------------ data phases
class DataManager:
    """Pre-builds one loader pair per phase and swaps them at phase epochs
    (train_imagenet_nv.py:545-598)."""

    def __init__(self, phases, args, device, dtype, log=None, tb=None):
        self.args, self.device, self.dtype, self.log, self.tb = args, device, dtype, log, tb
        self.phases = self.preload_phase_data(phases)
        self.trn_dl = self.val_dl = self.trn_smp = self.val_smp = None

    def set_epoch(self, epoch):
        cur = self.get_phase(epoch)
        if cur:
            self.set_data(cur)
        if hasattr(self.trn_smp, "set_epoch"):
            self.trn_smp.set_epoch(epoch)
        if hasattr(self.val_smp, "set_epoch"):
            self.val_smp.set_epoch(epoch)

    def get_phase(self, epoch):
        return next((p for p in self.phases if p["ep"] == epoch), None)

    def set_data(self, phase):
        if phase.get("keep_dl", False):
            if self.log:
                self.log.event(f"Batch size changed: {phase['bs']}")
            if self.tb:
                self.tb.log_size(phase["bs"])
            self.trn_dl.update_batch_size(phase["bs"])
            return
        if self.log:
            self.log.event(f"Dataset changed.\nImage size: {phase['sz']}\nBatch size: "
                           f"{phase['bs']}\nTrain Directory: {phase['trndir']}\nValidation "
                           f"Directory: {phase['valdir']}")
        if self.tb:
            self.tb.log_size(phase["bs"], phase["sz"])
        self.trn_dl, self.val_dl, self.trn_smp, self.val_smp = phase["data"]
        self.phases.remove(phase)

    def preload_phase_data(self, phases):
        for phase in phases:
            if not phase.get("keep_dl", False):
                trndir = phase.get("trndir", "")
                valdir = phase.get("valdir", trndir)
                phase["trndir"] = self.args.data + trndir + "/train"
                phase["valdir"] = self.args.data + valdir + "/validation"
                phase["data"] = self.preload_data(**phase)
        return phases

    def preload_data(self, ep, sz, bs, trndir, valdir, **kw):
        kw.pop("lr", None)
        val_bs = max(bs, 512) if sz == 128 else (max(bs, 256) if sz == 224 else max(bs, 128))
        if self.args.short_epoch:
            val_bs = bs
        n_train = self.args.synthetic_size or (12 if self.args.short_epoch else 64) * bs
        synthetic = self.args.data in ("synthetic", "")
        if not synthetic:
            # phases may name pre-resized copies (<data>-sz/160); use the full-size tree if absent
            if not os.path.isdir(trndir):
                trndir = os.path.join(self.args.data, "train")
            if not os.path.isdir(valdir):
                valdir = os.path.join(self.args.data, "validation")
            for d in (trndir, valdir):
                if not os.path.isdir(d):
                    raise FileNotFoundError(f"ImageNet directory {d} not found (pass 'synthetic' "
                                            "as DIR for the synthetic dataset)")
        return D.get_loaders(trndir, valdir, sz=sz, bs=bs, val_bs=val_bs,
                             workers=self.args.workers, rect_val=kw.get("rect_val", False),
                             min_scale=kw.get("min_scale", 0.08),
                             distributed=self.args.distributed, n_train=n_train,
                             n_val=(4 if self.args.short_epoch else 8) * val_bs,
                             device=self.device, dtype=self.dtype, synthetic=synthetic,
                             gpu_synthetic=synthetic and self.device.type == "cuda",
                             pad4=getattr(self.args, "pad4", False))


# ------------------------------------------------------------------------------------ run state
class Run:
    def __init__(self, args):
        self.args = args
        self.world = comm.world_size()
        self.rank = comm.rank()
        self.is_master = self.rank == 0
        self.fast = False          # set by main(): the fused / CompressedDDP / FlatSGD path
        self.tb = TensorboardLogger(args.logdir, is_master=self.is_master)
        self.log = FileLogger(args.logdir, is_master=self.is_master,
                              is_rank0=(args.local_rank or 0) == 0)


def save_checkpoint(run, epoch, model, best_top5, optimizer, is_best=False,
                    filename="checkpoint.pth.tar", extra=None):
    """``{'epoch', 'state_dict', 'best_top5', 'optimizer'}`` (+ optional extra keys, which older
    readers ignore) — train_imagenet_nv.py:663-669."""
    state = {"epoch": epoch + 1, "state_dict": model.state_dict(), "best_top5": best_top5,
             "optimizer": optimizer.state_dict()}
    if extra:
        state.update(extra)
    path = os.path.join(run.args.logdir or ".", filename)
    torch.save(state, path)
    if is_best and run.args.logdir:
        dst = os.path.join(run.args.logdir, "model_best.pth.tar")
        # the best checkpoint may already be written under that name (no self-copy)
        if not (os.path.exists(dst) and os.path.samefile(path, dst)):
            shutil.copyfile(path, dst)
    return path


def _fast_step(run, model, criterion, optimizer, eng):
    """The fused-path step closure (forward, loss, backward with overlapped compression, FlatSGD)
    wrapped in a :class:`~.graphs.StepGraph`, built once per run."""
    sg = getattr(run, "step_graph", None)
    if sg is not None:
        return sg
    args = run.args

    def body(inp, target):
        with torch.autocast(device_type=inp.device.type, dtype=h16(), cache_enabled=False):
            output = model(inp)
            loss = criterion(output.float(), target)
        (loss * args.loss_scale if args.fp16 else loss).backward()
        optimizer.step()
        last = getattr(criterion, "last_correct", None)
        return output.detach(), loss.detach(), last

    dev = next(model.parameters()).device
    run.step_graph = StepGraph(body, eng, optimizer, dev,
                               enabled=not getattr(args, "no_graph", False))
    return run.step_graph


def train(run, trn_loader, model, criterion, optimizer, scheduler, epoch, sync, master):
    args = run.args
    net_meter, timer = NetworkMeter(), TimeMeter()
    losses, top1, top5 = AverageMeter(), AverageMeter(), AverageMeter()
    model.train()
    fast = run.fast
    eng = getattr(model, "engine", None)
    acc = None                 # fast path: metrics summed on the device, read at print time
    t_mark, n_mark = time.perf_counter(), 0
    for i, (inp, target) in enumerate(trn_loader):
        if args.short_epoch and i > 10:
            break
        batch_num = i + 1
        timer.batch_start()
        scheduler.update_lr(epoch, batch_num, len(trn_loader))
        should_print = batch_num % args.print_freq == 0 or batch_num == len(trn_loader)
        step_fn = _fast_step(run, model, criterion, optimizer, eng) if fast else None
        if eng is not None:
            # per-bucket HIP-event timing makes a step eager; the same decision on every rank
            # (a rank running eagerly while the others replay would still pair its collectives,
            # but the logged numbers would describe a different step than the one timed), and
            # none while the step graph is on (the logged interval time is the replayed step's)
            eng.timing = should_print and (step_fn is None or not step_fn.enabled)
        if fast:
            # CompressedDDP: buckets compressed + exchanged during backward, the arena zeroed by
            # the next forward (no zero_grad); FlatSGD unscales a loss-scaled gradient itself.
            # The whole step runs as one replayed HIP graph once warm (train/graphs.py).
            output, loss, last = step_fn(inp, target)
        else:
            with torch.autocast(device_type=inp.device.type, dtype=torch.bfloat16,
                                enabled=args.bf16):
                output = model(inp)
                loss = criterion(output.float(), target)
            last = None
        if fast:
            pass
        elif args.fp16:
            scaled = loss * args.loss_scale
            model.zero_grad()
            scaled.backward()
            sync(model)
            model_params, master_params = master
            fp16util.model_grads_to_master_grads(model_params, master_params)
            for p in master_params:
                if p.grad is not None:
                    p.grad.data.mul_(1.0 / args.loss_scale)
            optimizer.step()
            fp16util.master_params_to_model_params(model_params, master_params)
        else:
            optimizer.zero_grad()
            loss.backward()
            sync(model)
            optimizer.step()
        if not fast:
            last = getattr(criterion, "last_correct", None)
        if last is not None:          # top-1/top-5 from the fused loss kernel (no topk pass)
            cs = last.sum(0)
            corr1, corr5 = cs[0:1], cs[1:2]
        else:
            corr1, corr5 = correct(output.data, target, topk=(1, 5))
        metrics = torch.cat([torch.tensor([float(inp.size(0))], device=loss.device),
                             loss.detach().float().reshape(1) * inp.size(0), corr1, corr5])
        if args.distributed and not fast:
            metrics = comm.sum_tensor(metrics)
        if fast:
            # no host sync and no collective per step (the reference all-reduces and reads the
            # metrics every step, train_imagenet_nv.py:421-424): accumulate this rank's sums on
            # the device and all-reduce the accumulated sums once per print interval — the same
            # totals, since summing over steps and over ranks commute
            acc = metrics.clone() if acc is None else acc.add_(metrics)
            timer.start = time.time()            # (data time only; step time per interval)
            if not should_print:
                run.tb.update_step_count(inp.size(0) * run.world)
                continue
            if args.distributed:
                acc = comm.sum_tensor(acc)
            batch_total, loss_sum, c1, c5 = acc.cpu().tolist()   # (waits for the GPU)
            acc = None
            # the interval's mean step time, GPU-complete (host time per step is not: the host
            # runs ahead of the device between syncs)
            now = time.perf_counter()
            timer.batch_time.update((now - t_mark) / (batch_num - n_mark), batch_num - n_mark)
            t_mark, n_mark = now, batch_num
        else:
            timer.batch_end()
            batch_total, loss_sum, c1, c5 = metrics.cpu().tolist()
        losses.update(loss_sum / batch_total, batch_total)
        top1.update(c1 * 100.0 / batch_total, batch_total)
        top5.update(c5 * 100.0 / batch_total, batch_total)
        if run.is_master and should_print:
            run.tb.log_memory()
            run.tb.log_trn_times(timer.batch_time.val, timer.data_time.val, inp.size(0))
            run.tb.log_trn_loss(losses.val, top1.val, top5.val)
            recv, sent = net_meter.update_bandwidth()
            run.tb.log("sizes/batch_total", batch_total)
            run.tb.log("net/recv_gbit", recv)
            run.tb.log("net/transmit_gbit", sent)
            if eng is not None:
                eng.read_overflow()
                run.tb.log_comm(eng.stats, eng.read_timings() if eng.timing else None)
            run.log.verbose(
                f"Epoch: [{epoch}][{batch_num}/{len(trn_loader)}]\tTime {timer.batch_time.val:.3f} "
                f"({timer.batch_time.avg:.3f})\tLoss {losses.val:.4f} ({losses.avg:.4f})\t"
                f"Acc@1 {top1.val:.3f} ({top1.avg:.3f})\tAcc@5 {top5.val:.3f} ({top5.avg:.3f})\t"
                f"Data {timer.data_time.val:.3f} ({timer.data_time.avg:.3f})\t"
                f"BW {recv:.3f} {sent:.3f}")
        run.tb.update_step_count(batch_total if not fast else inp.size(0) * run.world)
    if eng is not None:
        eng.timing = False
    return losses.avg, top1.avg, top5.avg


def distributed_predict(run, inp, target, model, criterion):
    """Uneven batches across ranks, a rank may hold none (train_imagenet_nv.py:523-542)."""
    bs = inp.size(0)
    dev = target.device
    loss = torch.zeros((), device=dev)
    c1 = torch.zeros(1, device=dev)
    c5 = torch.zeros(1, device=dev)
    valid = 0.0
    if bs:
        with torch.no_grad():
            output = model(inp)
            loss = criterion(output.float(), target).detach()
        valid = 1.0
        c1, c5 = correct(output, target, topk=(1, 5))
    metrics = torch.cat([torch.tensor([float(bs), valid], device=dev), loss.reshape(1).float(),
                         c1, c5])
    batch_total, valid_batches, reduced_loss, c1, c5 = comm.sum_tensor(metrics).cpu().tolist()
    reduced_loss = reduced_loss / max(valid_batches, 1)
    return c1 * 100.0 / max(batch_total, 1), c5 * 100.0 / max(batch_total, 1), reduced_loss, \
        batch_total


def validate(run, val_loader, model, criterion, epoch, start_time):
    args = run.args
    timer = TimeMeter()
    losses, top1, top5 = AverageMeter(), AverageMeter(), AverageMeter()
    if hasattr(model, "sync_buffers"):
        model.sync_buffers()              # collective, before any rank's (possibly empty) shard
    model.eval()
    t0 = time.time()
    for i, (inp, target) in enumerate(val_loader):
        if args.short_epoch and i > 10:
            break
        timer.batch_start()
        if args.distributed:
            a1, a5, loss, batch_total = distributed_predict(run, inp, target, model, criterion)
        else:
            with torch.no_grad():
                output = model(inp)
                loss = float(criterion(output.float(), target))
            batch_total = inp.size(0)
            a1, a5 = [float(a) for a in accuracy(output, target, topk=(1, 5))]
        timer.batch_end()
        losses.update(loss, batch_total)
        top1.update(a1, batch_total)
        top5.update(a5, batch_total)
        if run.is_master and ((i + 1) % args.print_freq == 0 or i + 1 == len(val_loader)):
            run.log.verbose(f"Test:  [{epoch}][{i + 1}/{len(val_loader)}]\tTime "
                            f"{timer.batch_time.val:.3f} ({timer.batch_time.avg:.3f})\tLoss "
                            f"{losses.val:.4f} ({losses.avg:.4f})\tAcc@1 {top1.val:.3f} "
                            f"({top1.avg:.3f})\tAcc@5 {top5.val:.3f} ({top5.avg:.3f})")
    run.tb.log_eval(top1.avg, top5.avg, time.time() - t0)
    run.tb.log("epoch", epoch)
    return top1.avg, top5.avg


def _bn_groups(model, params, wd):
    """``bnwd_optim_params`` without the D12 generator bug."""
    from .imagenet import bn_param_groups
    return bn_param_groups(model, wd, True)


def main(argv=None):
    args = get_parser().parse_args(argv)
    if args.local_rank is None:
        args.local_rank = int(os.environ.get("LOCAL_RANK", os.environ.get(
            "OMPI_COMM_WORLD_LOCAL_RANK", "0")))
    assert not (args.ddp and args.sparsification), "ddp and sparsification can't coexist"
    device = torch.device(args.device) if args.device else (
        torch.device("cuda", args.local_rank) if torch.cuda.is_available() else torch.device("cpu"))
    if device.type == "cuda":
        torch.cuda.set_device(device)
        torch.backends.cudnn.benchmark = True
    if args.distributed and not comm.is_dist():
        backend = args.dist_backend or ("nccl" if device.type == "cuda" else "gloo")
        dist.init_process_group(backend=backend, init_method=args.dist_url)
        assert comm.env_world_size() == dist.get_world_size()
    run = Run(args)
    log, tb = run.log, run.tb
    log.console(str(args))
    log.console(f"using seed {args.seed}")
    torch.manual_seed(args.seed)
    tb.log("sizes/world", run.world)

    model = getattr(R, args.arch)(bn0=args.init_bn0)
    # the MI355X path (default on a GPU): fused ResNet on the MFMA kernels, flat parameter /
    # gradient arenas, compression overlapped with backward (CompressedDDP), one fused SGD launch
    # (FlatSGD; --fp16 keeps its static loss scale, unscaled inside the SGD kernel). --no-fused
    # selects the reference's structure (torch layers, post-backward sync, torch SGD).
    run.fast = fast = device.type == "cuda" and not args.no_fused
    if fast:
        # --fp16 on the fused path: the fp16 build of the same MFMA kernels
        # (v_mfma_f32_16x16x32_f16, ops/_ext.py set_half), fp32 master weights with an fp16
        # mirror written by the SGD kernel, the static loss scale unscaled inside it
        # (train_imagenet_nv.py:410-428, fp16util.py:21-138). Without --fp16 the fused path
        # runs bf16 (no loss scale needed).
        set_half(bool(args.fp16))
        if args.fp16:
            log.console(f"--fp16: fused MFMA path in fp16, static loss scale {args.loss_scale}")
    if fast:
        lwnn.fuse_resnet(model)
    model = model.to(device)
    if device.type == "cuda":
        model = model.to(memory_format=torch.channels_last)
    if args.fp16 and not fast:
        model = fp16util.network_to_half(model)
    base_model = model
    sync = lambda m: None                                       # noqa: E731
    mc = float(args.momentum) if args.momentum_correction else 0.0
    if fast:
        if args.ddp:
            model = DistributedDataParallel(model, flat_params=True)
        elif args.sparsification:
            model = RandomKSparsifiedDDP(model, randk=args.randk, seed=args.seed,
                                         flat_params=True, dense_below=args.ef_dense_below,
                                         momentum_correction=mc)
        else:
            model = CompressedDDP(model, compress=args.compress, method=args.method,
                                  K=args.ratio, V=args.threshold, qstates=args.qstates,
                                  error_feedback=args.error_feedback, wire=args.wire,
                                  flat_params=True, dense_below=args.ef_dense_below,
                                  momentum_correction=mc)
    elif args.ddp:
        model = DistributedDataParallel(model)
    elif args.sparsification:
        model = RandomKSparsifiedDDP(model, randk=args.randk, seed=args.seed)
    elif args.overlap:
        model = CompressedDDP(model, compress=args.compress, method=args.method, K=args.ratio,
                              V=args.threshold, qstates=args.qstates,
                              error_feedback=args.error_feedback, wire=args.wire,
                              flat_params=False)
    else:
        if comm.is_dist():
            comm.broadcast_coalesced(list(model.state_dict().values()), 0)

        def sync(m):                                                # noqa: F811
            F.compressed_comm(m, args.compress, run.world, args.method, args.ratio,
                              args.threshold, args.qstates, error_feedback=args.error_feedback,
                              wire=args.wire)
    best_top5 = 93

    master = None
    if fast:
        from ..optim.flat_sgd import FlatSGD
        groups = _bn_groups(base_model, None, args.weight_decay) if args.no_bn_wd else \
            [{"params": [p for p in base_model.parameters() if p.requires_grad],
              "weight_decay": args.weight_decay}]
        om = 0.0 if mc > 0 else args.momentum        # DGC: the residual holds the velocity
        optimizer = FlatSGD(groups, model.arena, lr=0.0, momentum=om,
                            nesterov=om > 0, weight_decay=args.weight_decay,
                            grad_scale=1.0 / args.loss_scale if args.fp16 else 1.0)
        if mc > 0 and getattr(model, "engine", None) is not None:
            model.engine.set_mc_weight_decay(optimizer)   # decay enters the velocity
    elif args.fp16:
        master = fp16util.prep_param_lists(model)
        opt_params = _bn_groups(base_model, None, args.weight_decay) if args.no_bn_wd else None
        if opt_params is not None:   # map model params -> masters
            idx = {id(p): i for i, p in enumerate(master[0])}
            opt_params = [{"params": [master[1][idx[id(p)]] for p in g["params"]],
                           "weight_decay": g["weight_decay"]} for g in opt_params]
        else:
            opt_params = master[1]
    else:
        opt_params = _bn_groups(base_model, None, args.weight_decay) if args.no_bn_wd else \
            [p for p in model.parameters() if p.requires_grad]
    criterion = lwnn.FusedCrossEntropyLoss().to(device)
    if fast:
        pass
    elif args.momentum > 0:
        optimizer = torch.optim.SGD(opt_params, 0.0, momentum=args.momentum,
                                    weight_decay=args.weight_decay, nesterov=True)
    else:
        optimizer = torch.optim.SGD(opt_params, 0.0, weight_decay=args.weight_decay)

    phases = parse_phases(args.phases)
    dtype = h16() if fast else (torch.float16 if args.fp16 else torch.float32)
    args.pad4 = fast and bool(getattr(base_model, "_lw_stem_c4", False))
    dm = DataManager([copy.deepcopy(p) for p in phases if "bs" in p], args, device, dtype,
                     log, tb)
    scheduler = Scheduler(optimizer, [copy.deepcopy(p) for p in phases if "lr" in p], log, tb,
                          args.momentum)

    if args.resume:
        ckpt = torch.load(args.resume, map_location=device, weights_only=True)
        model.load_state_dict(adapt_state_dict(ckpt["state_dict"], model))
        args.start_epoch = ckpt["epoch"]
        best_top5 = ckpt["best_top5"]
        if not args.evaluate:            # eval-only needs the weights, not the optimizer state
            optimizer.load_state_dict(ckpt["optimizer"])
        if "scheduler" in ckpt:
            scheduler.load_state_dict(ckpt["scheduler"])
        if "compression" in ckpt and hasattr(model, "load_compression_state"):
            model.load_compression_state(ckpt["compression"])
            ef = getattr(model.engine, "ef", None)
            if ef is not None:
                log.console(f"EF residual restored: |e|={float(ef.double().norm()):.9e}")
        log.console(f"resumed from {args.resume} at epoch {args.start_epoch}")

    start_time = datetime.now()
    if args.evaluate:
        dm.set_epoch(args.start_epoch)
        return validate(run, dm.val_dl, model, criterion, 0, start_time)

    if args.distributed:
        log.console("Syncing machines before training")
        comm.sum_tensor(torch.tensor([1.0], device=device))

    log.event("~~epoch\thours\ttop1\ttop5\n")
    end_epoch = scheduler.tot_epochs if args.epochs is None else min(scheduler.tot_epochs,
                                                                     args.start_epoch + args.epochs)
    # phases before start_epoch must still be applied (resume mid-schedule)
    for e in range(0, args.start_epoch):
        if dm.get_phase(e):
            dm.set_epoch(e)
    top1 = top5 = 0.0
    for epoch in range(args.start_epoch, end_epoch):
        dm.set_epoch(epoch)
        train(run, dm.trn_dl, model, criterion, optimizer, scheduler, epoch, sync, master)
        sg = getattr(run, "step_graph", None)
        if sg is not None:
            log.event(f"HIP-graph step replays so far: {sg.replays} "
                      f"({'active' if sg.active() else 'eager'})")
        top1, top5 = validate(run, dm.val_dl, model, criterion, epoch, start_time)
        hours = (datetime.now() - start_time).total_seconds() / 3600.0
        log.event(f"~~{epoch}\t{hours:.5f}\t\t{top1:.3f}\t\t{top5:.3f}\n")
        is_best = top5 > best_top5
        best_top5 = max(top5, best_top5)
        # every rank takes part: the error-feedback residuals are per rank (a collective
        # gathers them to the checkpoint writer); the BN buffers saved are rank 0's, synced
        if hasattr(model, "sync_buffers"):
            model.sync_buffers()
        comp = model.compression_state() if args.extra_ckpt and \
            hasattr(model, "compression_state") else None
        if args.local_rank == 0 and run.is_master:
            extra = None
            if args.extra_ckpt:
                extra = {"scheduler": scheduler.state_dict()}
                if comp is not None:
                    extra["compression"] = comp
                    if comp.get("ef_per_rank") is not None:
                        log.console("EF residual saved: |e|="
                                    f"{float(comp['ef_per_rank'][run.rank].double().norm()):.9e}")
            if is_best:
                save_checkpoint(run, epoch, model, best_top5, optimizer, is_best=True,
                                filename="model_best.pth.tar", extra=extra)
            phase = dm.get_phase(epoch)
            if phase:
                save_checkpoint(run, epoch, model, best_top5, optimizer,
                                filename=f"sz{phase['bs']}_checkpoint.path.tar", extra=extra)
            save_checkpoint(run, epoch, model, best_top5, optimizer, filename="checkpoint.pth.tar",
                            extra=extra)
    tb.close()
    return top1, top5


if __name__ == "__main__":
    main(sys.argv[1:])
