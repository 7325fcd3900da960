"""Job launcher (reference ``IMAGENET/train.py``): picks the progressive-resizing schedule for the
machine count and starts one training process per GPU.

    python -m IMAGENET.train --machines 1 --nproc_per_node 8 -c layerwise --method Topk -K 0.001

Single node: processes are spawned locally (torchrun contract, RCCL over xGMI). Multi-node: the
per-node ``torchrun`` command lines are printed (``--master_addr`` required) — AWS provisioning,
EBS volume mounting and EFA/MPI plumbing of the reference are out of scope on MI355X nodes.
Unlike the reference compression flags ARE forwarded to the workers.
"""
from __future__ import annotations

import argparse
import os
import sys

from ..utils.launch import launch_local, node_commands, ring_env
from .schedules import schedules

WORKER = "IMAGENET/training/train_imagenet_nv.py"


def get_parser():
    p = argparse.ArgumentParser(description="launch compressed-gradient ImageNet training")
    p.add_argument("--name", type=str, default="imagenet")
    p.add_argument("--machines", type=int, default=1, choices=sorted(schedules))
    p.add_argument("--nproc_per_node", type=int, default=8)
    p.add_argument("--master_addr", type=str, default="127.0.0.1")
    p.add_argument("--master_port", type=int, default=None)
    p.add_argument("--data", type=str, default="synthetic")
    p.add_argument("--logdir", type=str, default=None)
    p.add_argument("--simple_ring_setup", action="store_true")
    p.add_argument("--no_op", action="store_true", help="run the environment test instead")
    p.add_argument("--print_only", action="store_true")
    p.add_argument("--log_all_workers", action="store_true")
    p.add_argument("--cuda_debug", action="store_true",
                   help="AMD_SERIALIZE_KERNEL=3 NCCL_DEBUG=INFO")
    p.add_argument("--timeout", type=float, default=None)
    return p


def build_worker_args(args, extra):
    logdir = args.logdir or os.path.join("runs", args.name)
    wa = [WORKER, args.data, "--logdir", logdir, "--distributed", "--init-bn0", "--no-bn-wd",
          "--name", args.name, "--phases", {1: "one_machine", 2: "two_machines",
                                            4: "four_machines", 8: "eight_machines",
                                            16: "sixteen_machines"}[args.machines]]
    if args.log_all_workers:
        wa += ["--log_all_workers", "1"]
    return wa + list(extra)


def main(argv=None):
    args, extra = get_parser().parse_known_args(argv)
    env = ring_env(args.machines, args.nproc_per_node, args.simple_ring_setup)
    env["OMP_NUM_THREADS"] = env.get("OMP_NUM_THREADS", "1")
    if args.cuda_debug:
        env.update(AMD_SERIALIZE_KERNEL="3", NCCL_DEBUG="INFO")
    if args.no_op:
        wa = ["-c", "import torch, torch.distributed as d, os; d.init_process_group("
                    "'nccl' if torch.cuda.is_available() else 'gloo'); "
                    "print('rank', d.get_rank(), 'of', d.get_world_size(), 'ok'); "
                    "d.destroy_process_group()"]
    else:
        wa = build_worker_args(args, extra)
    if args.machines > 1 or args.print_only:
        for cmd in node_commands(wa[0], wa[1:], args.machines, args.nproc_per_node,
                                 args.master_addr, args.master_port or 29500):
            print(" ".join(f"{k}='{v}'" for k, v in env.items()), cmd)
        return 0
    return launch_local(wa, args.nproc_per_node, args.master_addr, args.master_port,
                        extra_env=env, timeout=args.timeout)


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
