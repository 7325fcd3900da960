"""CIFAR-10 entry point with the reference CLI (``CIFAR10/dawn.py:8-20, 98-155``).

    python -m CIFAR10.dawn -m tcp://127.0.0.1:2222 -r 0 -w 2 -n Resent9 -c layerwise \
        --method Topk -K 0.01

Recipe (``dawn.py:105-148``): 24 epochs (40 for Randomk / Thresholdv), batch 512 per rank,
``PiecewiseLinear([0, 5, E], [0, 0.4, 0])`` evaluated at ``step / len(train_batches)`` and divided
by the batch size (per-sample LR with a summed loss), SGD with ``wd = 5e-4 · bs`` and Nesterov
momentum only when ``--momentum > 0``, crop / flip / cutout augmentation redrawn every epoch.
Writes ``logs.tsv`` (``epoch\\thours\\ttop1Accuracy``) to ``--log_dir``.

Added flags (all optional): ``--epochs``, ``--error_feedback``, ``--wire``, ``--synthetic``,
``--max_batches`` (debug), ``--dtype``, ``--backend``, ``--full_data`` (every rank iterates the whole
training set, as the reference does — by default each rank sees its 1/W shard, D16), ``--device``.

Device placement: each rank binds to ``cuda:LOCAL_RANK`` (``rank % device_count`` without a
launcher-provided local rank), so ``-w 8`` on one node puts one rank on each GPU. The reference
puts every rank on ``cuda:0`` (``CIFAR10/torch_backend.py:8``).
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

from ..data import cifar as D
from ..models.cifar import build_network
from ..models.graph import SGD, trainable_params
from ..utils.logging import PiecewiseLinear, TableLogger, Timer, TSVLogger
from .cifar import train


def get_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="layer-wise / entire-model compressed CIFAR-10")
    p.add_argument("--data_dir", type=str, default="./data")
    p.add_argument("--log_dir", type=str, default=".")
    p.add_argument("--master_address", "-m", type=str, default="127.0.0.1")
    p.add_argument("--rank", "-r", type=int, default=0)
    p.add_argument("--world_size", "-w", type=int, default=2)
    p.add_argument("--network", "-n", type=str, default="resnet9")
    p.add_argument("--compress", "-c", type=str, default="none")
    p.add_argument("--method", type=str, default="none")
    p.add_argument("--ratio", "-K", type=float, default=0.5)
    p.add_argument("--threshold", "-V", type=float, default=0.001)
    p.add_argument("--qstates", "-Q", type=int, default=255)
    p.add_argument("--momentum", type=float, default=0.0)
    # additions
    p.add_argument("--epochs", type=int, default=None)
    p.add_argument("--batch_size", type=int, default=512)
    p.add_argument("--error_feedback", action="store_true")
    p.add_argument("--wire", default="auto", choices=["auto", "sparse", "sparse-exact", "sparse-capped", "dense", "indexfree", "qrs"])
    p.add_argument("--synthetic", action="store_true")
    p.add_argument("--n_train", type=int, default=50000)
    p.add_argument("--n_test", type=int, default=10000)
    p.add_argument("--max_batches", type=int, default=None)
    p.add_argument("--backend", type=str, default=None)
    p.add_argument("--full_data", action="store_true",
                   help="every rank iterates the full training set (reference behaviour)")
    p.add_argument("--shard_data", action="store_true",
                   help="(default; kept for old command lines) each rank sees 1/W of the data")
    p.add_argument("--device", type=str, default=None)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--ef_dense_below", type=int, default=0,
                   help="(opt-in) Top-K / Random-K: tensors of at most this many elements are "
                        "sent whole (profiles/r4/ef_root_cause.md)")
    p.add_argument("--momentum_correction", action="store_true",
                   help="(opt-in, needs --error_feedback and --momentum) DGC momentum correction "
                        "+ factor masking: the velocity is accumulated before compression and the "
                        "optimizer runs without momentum")
    p.add_argument("--no_fused", action="store_true",
                   help="the reference's structure: torch layers, post-backward sync, torch SGD")
    return p


def main(argv=None):
    args = get_parser().parse_args(argv)
    from ..parallel.comm import bind_rank_device
    device = bind_rank_device(args.rank, args.device)
    torch.manual_seed(args.seed)
    np.random.seed(args.seed + args.rank)

    dataset = D.synthetic_cifar10(args.n_train, args.n_test, args.seed) if args.synthetic else \
        D.cifar10(args.data_dir, n_train=args.n_train, n_test=args.n_test)
    epochs = args.epochs or (40 if args.method in ("Randomk", "Thresholdv") else 24)
    lr_schedule = PiecewiseLinear([0, 5, epochs], [0, 0.4, 0])
    bs = args.batch_size
    model = build_network(args.network)
    # MI355X path (default on a GPU): fused BN+ReLU, every conv / Linear on the MFMA kernels,
    # bf16 autocast + channels_last, CompressedDDP (compression overlapped with backward) and
    # the fused flat-arena SGD; --no_fused keeps the reference's structure.
    fast = device.type == "cuda" and not args.no_fused
    if fast:
        from ..ops import nn as lwnn
        from ..ops.conv import fuse_convs
        from ..ops.gemm import fuse_linears
        lwnn.fuse_graph_network(model)
        fuse_convs(model)
        fuse_linears(model)
    model = model.to(device)
    if fast:
        model = model.to(memory_format=torch.channels_last)

    timer = Timer(synch=torch.cuda.synchronize if device.type == "cuda" else None)
    train_x = D.transpose(D.normalise(D.pad(dataset["train"]["data"], 4)))
    test_x = D.transpose(D.normalise(dataset["test"]["data"]))
    shard = (0, 1) if args.full_data else (args.rank, args.world_size)
    train_batches = D.GPUBatches(torch.from_numpy(np.ascontiguousarray(train_x)).to(device),
                                 torch.as_tensor(dataset["train"]["labels"]).to(device), bs,
                                 shuffle=True, augment=True, drop_last=True, shard=shard,
                                 seed=args.seed, channels_last=fast)
    test_batches = D.GPUBatches(torch.from_numpy(np.ascontiguousarray(test_x)).to(device),
                                torch.as_tensor(dataset["test"]["labels"]).to(device), bs,
                                shuffle=False, channels_last=fast)
    print(f"Finished preprocessing in {timer():.2f} seconds")

    def lr(step):
        return lr_schedule(step / max(len(train_batches), 1)) / bs

    net = model
    optimizer_cls = torch.optim.SGD
    from ..parallel import comm as _comm
    owns_pg = not _comm.is_dist()            # this CLI created the process group (and ends it)
    if fast:
        from ..optim.flat_sgd import FlatSGD
        from ..parallel.ddp import CompressedDDP
        from .cifar import init_distributed
        init_distributed(args.master_address, args.world_size, args.rank, args.backend)
        model = CompressedDDP(net, compress=args.compress, method=args.method, K=args.ratio,
                              V=args.threshold, qstates=args.qstates,
                              error_feedback=args.error_feedback, wire=args.wire,
                              flat_params=True, dense_below=args.ef_dense_below,
                              momentum_correction=args.momentum if args.momentum_correction
                              else 0.0)
        arena = model.arena

        def optimizer_cls(weights, **kw):               # noqa: F811
            return FlatSGD(weights, arena, **kw)
    if args.momentum > 0 and not (fast and args.momentum_correction):
        opt = SGD(trainable_params(net), lr=lr, momentum=args.momentum, weight_decay=5e-4 * bs,
                  nesterov=True, optimizer=optimizer_cls)
    else:
        opt = SGD(trainable_params(net), lr=lr, weight_decay=5e-4 * bs, optimizer=optimizer_cls)

    tsv = TSVLogger()
    train(model, opt, train_batches, test_batches, epochs, args.master_address, args.world_size,
          args.rank, loggers=(TableLogger(), tsv), timer=timer, test_time_in_total=False,
          compress="none" if fast else args.compress, method=args.method, K=args.ratio,
          V=args.threshold, qstates=args.qstates, backend=args.backend,
          error_feedback=args.error_feedback, wire=args.wire, max_batches=args.max_batches,
          autocast=torch.bfloat16 if fast else None)
    sg = getattr(model, "_lw_step_graph", None)
    if sg is not None:
        print(f"HIP-graph step: {sg.replays} replays, {sg.captures} capture(s), "
              f"{'active' if sg.enabled else 'eager'}", flush=True)
    os.makedirs(os.path.expanduser(args.log_dir), exist_ok=True)
    with open(os.path.join(os.path.expanduser(args.log_dir), "logs.tsv"), "w") as f:
        f.write(str(tsv))
    from ..parallel import comm
    if comm.is_dist() and owns_pg:
        comm.dist.barrier()
        comm.shutdown_native()
        comm.dist.destroy_process_group()
    return tsv


if __name__ == "__main__":
    main(sys.argv[1:])
