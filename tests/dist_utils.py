"""Helpers to run a function on N gloo ranks (CPU) and collect per-rank results."""
import os
import pickle
import socket
import tempfile
import traceback

import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fn, outdir, args):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    res = None
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        res = ("ok", fn(rank, world, *args))
    except Exception:  # noqa: BLE001
        res = ("err", traceback.format_exc())
    finally:
        with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
            pickle.dump(res, f)           # our own files, written by this test
        if dist.is_initialized():
            dist.destroy_process_group()


def run_world(fn, world=2, args=()):
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, port, fn, d, args), nprocs=world,
                           start_method="spawn", join=True)
        out = []
        for r in range(world):
            with open(os.path.join(d, f"r{r}.pkl"), "rb") as f:
                status, val = pickle.load(f)
            if status != "ok":
                raise AssertionError(f"rank {r} failed:\n{val}")
            out.append(val)
    return out
