"""Launch orchestration: single-node multi-process launcher, env helpers, ring-order
builders and a safe text encoding for configs.

The reference drives AWS instances through ``ncluster`` and starts workers with
``torch.distributed.launch`` or ``mpirun`` over EFA (``IMAGENET/train.py:290-449``,
``IMAGENET/util.py``). On an MI355X node the equivalent is one process per GPU on one host: this
module spawns them with ``RANK`` / ``LOCAL_RANK`` / ``WORLD_SIZE`` / ``MASTER_ADDR`` /
``MASTER_PORT`` set (torchrun's contract), or emits the per-node command lines for multi-node runs.
RCCL detects the xGMI topology itself, so the NCCL ring strings are kept only as a multi-node aid.
"""
from __future__ import annotations

import base64
import json
import os
import random
import re
import signal
import socket
import string
import subprocess
import sys
import time
from typing import Dict, List, Optional, Sequence


def is_set(name: str) -> bool:
    """Env flag set to anything but missing / 0 / false (``util.py:12-16``)."""
    return os.environ.get(name, "0").lower() not in ("0", "false", "")


def random_id(k: int = 3) -> str:
    return "".join(random.choices(string.ascii_lowercase + string.digits, k=k))


def environment_snapshot() -> Dict[str, str]:
    """What ``util.log_environment`` records: NCCL/RCCL/HIP/PATH/LD/OMP variables + versions."""
    import torch
    snap = {k: v for k, v in os.environ.items()
            if re.match(r"^(NCCL|RCCL|HIP|ROCM|HSA|CUDA|PATH|LD|USER|PWD|OMP)", k)}
    snap["pytorch_version"] = torch.__version__
    snap["hip_version"] = str(getattr(torch.version, "hip", None))
    return snap


def log_environment(logger=None) -> Dict[str, str]:
    snap = environment_snapshot()
    if logger is not None:
        for k, v in sorted(snap.items()):
            logger.console(f"env {k}={v}")
    return snap


def ossystem(cmd: str, shell: bool = True) -> str:
    p = subprocess.run(cmd, shell=shell, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    return p.stdout.decode("utf-8", "replace")


def text_encode(obj) -> str:
    """Config → ASCII (base64 JSON). Replaces ``text_pickle``: nothing is ever unpickled."""
    return base64.b64encode(json.dumps(obj).encode()).decode("ascii")


def text_decode(s: str):
    if not s:
        return None
    return json.loads(base64.b64decode(s).decode())


def format_env(**kw) -> str:
    return " ".join(f"{k}={v}" for k, v in kw.items())


def format_env_export(**kw) -> str:
    """``export K=V`` chain for shell command prefixes (``util.format_env_export``)."""
    return "; ".join(f"export {k}={v}" for k, v in kw.items())


def get_nccl_params(num_tasks: int, num_gpus: int, simple: bool = False) -> str:
    """Collective tuning environment as one ``K=V ...`` string (``train.py:159-187``); RCCL reads
    the same variable names."""
    return format_env(**ring_env(num_tasks, num_gpus, simple))


def setup_mpi(hosts: Sequence[str], slots: int, path: str = "hosts.slots",
              env: Optional[Dict[str, str]] = None) -> str:
    """Write an MPI hostfile (one ``host slots=N`` line per node, ``util.setup_mpi``) and return the
    ``mpirun`` prefix that exports the rank variables the worker reads (``train.py:412-416``).
    Passwordless ssh between the nodes is assumed to be configured by the cluster (the reference's
    key exchange is AWS-specific)."""
    with open(path, "w") as f:
        for h in hosts:
            f.write(f"{h} slots={slots}\n")
    exports = " ".join(f"-x {k}={v}" for k, v in (env or {}).items())
    n = len(hosts) * slots
    return (f"mpirun -n {n} -N {slots} --hostfile {path} --bind-to none {exports} "
            "-x MASTER_ADDR -x MASTER_PORT").strip()


def run_parallel(fns: Sequence, max_workers: Optional[int] = None) -> list:
    """Run callables concurrently and return their results in order (``util.run_parallel``)."""
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=max_workers or max(1, len(fns))) as ex:
        return list(ex.map(lambda f: f(), fns))


def mount_imagenet(path: str, required=("train", "validation")) -> str:
    """Check that an ImageNet-layout tree is present on this node (the reference attached and
    mounted an EBS volume per task, ``train.py:227-287``; MI355X nodes read local NVMe / shared
    storage — stage it with ``IMAGENET/tools/replicate_imagenet.py``)."""
    missing = [d for d in required if not os.path.isdir(os.path.join(path, d))]
    if missing:
        raise FileNotFoundError(f"{path} lacks {missing}; stage the dataset first "
                                "(IMAGENET/tools/replicate_imagenet.py)")
    return path


# ----------------------------------------------------------------------------- ring orders
def build_ring_order(machine_order: Sequence[int], gpu_order: Sequence[int]) -> str:
    gpus = list(gpu_order)
    return " ".join(str(m * len(gpus) + g) for m in machine_order for g in gpus)


def get_skip_order(size: int) -> List[int]:
    if size == 4:
        return [0, 2, 1, 3]
    step = 5 if size == 16 else 3
    return [(i * step) % size for i in range(size)]


def get_rings(num_tasks: int, num_gpus: int) -> str:
    """Forward + reverse rings, plus two "skip" rings for >= 4 nodes of 8 GPUs
    (``train.py:171-192``). Formatted for ``NCCL_RINGS`` (RCCL honours the same variable)."""
    ring = build_ring_order(range(num_tasks), range(num_gpus))
    rev = build_ring_order(reversed(range(num_tasks)), reversed(range(num_gpus)))
    rings = [ring, rev]
    if num_tasks >= 4 and num_gpus == 8:
        assert num_tasks % 4 == 0
        sm = get_skip_order(num_tasks)
        rings += [build_ring_order(sm, [3, 2, 1, 0, 7, 6, 5, 4]),
                  build_ring_order(list(reversed(sm)), get_skip_order(num_gpus))]
    return " | ".join(rings)


def ring_env(num_tasks: int, num_gpus: int, simple: bool = False) -> Dict[str, str]:
    if num_tasks <= 1:
        return {"NCCL_DEBUG": "VERSION"}
    if simple:
        return {"NCCL_MIN_NRINGS": "16", "NCCL_MAX_NRINGS": "16"}
    return {"NCCL_RINGS": get_rings(num_tasks, num_gpus), "NCCL_SINGLE_RING_THRESHOLD": "10"}


# ----------------------------------------------------------------------------- local launcher
def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_local(argv: Sequence[str], nproc: int, master_addr: str = "127.0.0.1",
                 master_port: Optional[int] = None, node_rank: int = 0, nnodes: int = 1,
                 extra_env: Optional[Dict[str, str]] = None, timeout: Optional[float] = None,
                 log_dir: Optional[str] = None) -> int:
    """Start ``nproc`` copies of ``python <argv...>`` (one per GPU) and wait. A failing rank
    terminates the others; the first non-zero exit code is returned."""
    port = master_port or free_port()
    world = nproc * nnodes
    procs = []
    for lr in range(nproc):
        env = dict(os.environ)
        env.update(extra_env or {})
        env.update(RANK=str(node_rank * nproc + lr), LOCAL_RANK=str(lr), WORLD_SIZE=str(world),
                   LOCAL_WORLD_SIZE=str(nproc), MASTER_ADDR=master_addr, MASTER_PORT=str(port))
        out = None
        if log_dir:
            os.makedirs(log_dir, exist_ok=True)
            out = open(os.path.join(log_dir, f"rank{node_rank * nproc + lr}.log"), "w")
        procs.append((subprocess.Popen([sys.executable, *argv], env=env, stdout=out,
                                       stderr=subprocess.STDOUT if out else None,
                                       start_new_session=True), out))
    t0 = time.time()
    rc = 0
    try:
        alive = list(range(nproc))
        while alive:
            for i in list(alive):
                code = procs[i][0].poll()
                if code is not None:
                    alive.remove(i)
                    if code != 0 and rc == 0:
                        rc = code
                        for j in alive:
                            os.killpg(procs[j][0].pid, signal.SIGTERM)
            if timeout and time.time() - t0 > timeout:
                for j in alive:
                    os.killpg(procs[j][0].pid, signal.SIGKILL)
                return 124
            time.sleep(0.05)
    finally:
        for _, f in procs:
            if f:
                f.close()
    return rc


def node_commands(script: str, script_args: Sequence[str], nnodes: int, nproc: int,
                  master_addr: str, master_port: int = 29500) -> List[str]:
    """torchrun command line for every node of a multi-node run."""
    return [" ".join([sys.executable, "-m", "torch.distributed.run", f"--nnodes={nnodes}",
                      f"--nproc-per-node={nproc}", f"--node-rank={r}",
                      f"--master-addr={master_addr}", f"--master-port={master_port}", script,
                      *script_args]) for r in range(nnodes)]
