"""Collective helpers over ``torch.distributed`` (RCCL on GPU via the "nccl" backend, gloo on CPU).

The reference issues one *blocking* collective per parameter tensor (``CIFAR10/core.py:218``,
``train_imagenet_nv.py:298, 385``). Here every collective is asynchronous on
the backend's own stream and operates on a whole bucket; the caller keeps the handle and
``wait()``s it only when the result is consumed, which on RCCL makes the *compute stream* wait on an
event rather than blocking the host.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

dist = dist  # re-exported for callers that need ReduceOp / backend queries


def inject_fault(kind: str, rank_: int) -> bool:
    """Test hook: ``LWAAAI_INJECT_FAULT=<kind>:<rank>`` (kinds: ``capture`` — the step-graph
    capture raises, ``native_init`` — the native RCCL init raises before joining) fires on that
    rank only."""
    spec = os.environ.get("LWAAAI_INJECT_FAULT", "")
    return spec == f"{kind}:{int(rank_)}"


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized()


def world_size(group=None) -> int:
    return dist.get_world_size(group) if is_dist() else 1


def rank(group=None) -> int:
    return dist.get_rank(group) if is_dist() else 0


def env_world_size() -> int:
    """``dist_utils.env_world_size`` (IMAGENET/training/dist_utils.py:27), defaulting to 1."""
    return int(os.environ.get("WORLD_SIZE", "1"))


def env_rank() -> int:
    return int(os.environ.get("RANK", "0"))


def env_local_rank() -> Optional[int]:
    """``LOCAL_RANK`` (torchrun) or ``OMPI_COMM_WORLD_LOCAL_RANK`` (mpirun), None if neither."""
    for k in ("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK"):
        if os.environ.get(k, "") != "":
            return int(os.environ[k])
    return None


def rank_device_index(rank: int, n_devices: int, local_rank: Optional[int] = None) -> int:
    """The GPU a rank binds to: its launcher-provided local rank when there is one, otherwise
    ``rank % n_devices`` (one process per GPU on every node). The reference puts every rank on
    ``cuda:0`` (``CIFAR10/torch_backend.py:8``); the ImageNet script uses ``local_rank``
    (``train_imagenet_nv.py:160``)."""
    if n_devices <= 0:
        raise ValueError("no GPU to bind to")
    idx = local_rank if local_rank is not None else int(rank)
    return idx % n_devices


def bind_rank_device(rank: int, requested: Optional[str] = None) -> torch.device:
    """Pick and select this rank's device: ``requested`` verbatim when given (``--device``),
    otherwise ``cuda:<rank_device_index>`` when a GPU is visible, else the CPU."""
    if requested:
        dev = torch.device(requested)
    elif torch.cuda.is_available():
        dev = torch.device("cuda", rank_device_index(rank, torch.cuda.device_count(),
                                                     env_local_rank()))
    else:
        dev = torch.device("cpu")
    if dev.type == "cuda":
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        torch.cuda.set_device(dev)
    return dev


def agree(ok: bool, group=None, device=None) -> bool:
    """All-rank AND of a local flag (one tiny all-reduce; ``True`` without a process group), so
    a fallback decision — graph capture, native communicator — is taken by every rank or none."""
    if not is_dist() or world_size(group) == 1:
        return bool(ok)
    dev = torch.device(device) if device is not None and \
        dist.get_backend(group) == "nccl" else torch.device("cpu")
    if dist.get_backend(group) == "nccl" and dev.type != "cuda":
        dev = torch.device("cuda", torch.cuda.current_device())
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


class _Done:
    def wait(self):
        return True

    def is_completed(self):
        return True


def all_reduce(t: torch.Tensor, group=None, async_op: bool = True, op=None):
    if not is_dist() or world_size(group) == 1 and t.device.type == "cpu":
        return _Done()
    op = op if op is not None else dist.ReduceOp.SUM
    return dist.all_reduce(t, op=op, group=group, async_op=async_op) or _Done()


def all_gather(out: torch.Tensor, inp: torch.Tensor, group=None, async_op: bool = True):
    if not is_dist() or world_size(group) == 1 and inp.device.type == "cpu":
        out.copy_(inp)
        return _Done()
    return dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op) or _Done()


def _bcast_uid(uid: torch.Tensor, group, dev) -> torch.Tensor:
    if world_size(group) <= 1:
        return uid
    t = uid.to(dev)
    src = dist.get_global_rank(group, 0) if group is not None else 0
    dist.broadcast(t, src=src, group=group)
    return t.cpu()


class NativeRccl:
    """Direct RCCL communicator (``csrc/rccl.cpp``) for the stream-ordered, graph-capturable
    bucket collectives: calls are enqueued on the caller's current HIP stream and return
    :class:`_Done` (nothing to wait for on the host; later work on that stream is ordered after
    them). Built collectively over an initialised ``nccl`` process group: rank 0's unique id is
    broadcast through it, then every rank joins with ``ncclCommInitRank``."""

    def __init__(self, group=None, device=None, uid: Optional[torch.Tensor] = None):
        from ..ops._ext import load_main as load
        self.lib = load()
        self.world = world_size(group)
        self.rank = rank(group)
        self.handle = 0
        dev = torch.device(device) if device is not None else \
            torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        if uid is None:       # (given: already broadcast by the caller)
            uid = self.lib.rccl_unique_id() if self.rank == 0 else \
                torch.zeros(128, dtype=torch.uint8)
            uid = _bcast_uid(uid, group, dev)
        if inject_fault("native_init", self.rank):
            # test hook: this rank fails BEFORE joining ncclCommInitRank, so its peers are left
            # waiting inside their (non-blocking) init until the deadline aborts it
            raise RuntimeError("injected native init failure (LWAAAI_INJECT_FAULT)")
        self.handle = int(self.lib.rccl_init(uid, self.world, self.rank, dev.index or 0,
                                             init_timeout()))

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor):
        self.lib.rccl_all_gather(self.handle, inp, out)
        return _Done()

    def all_reduce(self, t: torch.Tensor, op: str = "sum"):
        self.lib.rccl_all_reduce(self.handle, t, {"sum": 0, "max": 1, "min": 2}[op])
        return _Done()

    def broadcast(self, t: torch.Tensor, src: int = 0):
        self.lib.rccl_broadcast(self.handle, t, src)
        return _Done()

    def send_recv(self, sends, send_peers, recvs, recv_peers, key=None):
        """Every send / receive of the lists in one RCCL group (``csrc/rccl.cpp
        rccl_send_recv``); ``key`` is for stand-ins that must know what the peers would send."""
        self.lib.rccl_send_recv(self.handle, list(sends), [int(p) for p in send_peers],
                                list(recvs), [int(p) for p in recv_peers])
        return _Done()

    def all_to_all(self, send: torch.Tensor, recv: torch.Tensor):
        self.lib.rccl_all_to_all(self.handle, send, recv)
        return _Done()

    def reduce_scatter(self, send: torch.Tensor, recv: torch.Tensor, op: str = "sum"):
        self.lib.rccl_reduce_scatter(self.handle, send, recv, {"sum": 0, "max": 1, "min": 2}[op])
        return _Done()

    def start_watchdog(self, timeout_s: float, action: int = 0) -> "Watchdog":
        """Deadline + asynchronous-error watchdog on this communicator (``csrc/rccl.cpp``)."""
        self.watch = Watchdog(self.handle, self.device, timeout_s, action)
        return self.watch

    def close(self) -> None:
        """Stop the watchdog and free the communicator locally (``ncclCommAbort``: it involves no
        peer, so a teardown in any rank order cannot block)."""
        w = getattr(self, "watch", None)
        if w is not None:
            w.close()
            self.watch = None
        if self.handle:
            self.lib.rccl_abort(self.handle)
            self.handle = 0


class C10dP2P:
    """``send_recv`` over c10d point-to-point (``dist.batch_isend_irecv``: gloo on the CPU, or
    the nccl process group when the native communicator is off) with the native communicator's
    signature; transfers to this rank itself are local copies. Blocking: returns once every
    transfer has completed."""

    def __init__(self, group=None):
        self.group = group
        self.rank = rank(group)

    def _global(self, peer: int) -> int:
        return dist.get_global_rank(self.group, peer) if self.group is not None else int(peer)

    def send_recv(self, sends, send_peers, recvs, recv_peers, key=None):
        ops = []
        mine = [t for t, p in zip(sends, send_peers) if int(p) == self.rank]
        into = [t for t, p in zip(recvs, recv_peers) if int(p) == self.rank]
        if len(mine) != len(into):
            raise ValueError("send_recv: sends to self and receives from self do not pair up")
        for a, b in zip(mine, into):
            b.copy_(a)
        for t, p in zip(sends, send_peers):
            if int(p) != self.rank and t.numel():
                ops.append(dist.P2POp(dist.isend, t.contiguous(), self._global(p), self.group))
        for t, p in zip(recvs, recv_peers):
            if int(p) != self.rank and t.numel():
                ops.append(dist.P2POp(dist.irecv, t, self._global(p), self.group))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        return _Done()


class Watchdog:
    """Host thread that fails a run loudly instead of letting it hang (``csrc/rccl.cpp``).

    The native RCCL calls bypass c10d and therefore its ProcessGroup watchdog. This one:

    * polls ``ncclCommGetAsyncError``;
    * checks that the step completion event recorded by :meth:`mark` (once per step, outside
      graph capture) completes within ``timeout_s``.

    When either check fails:

    * ``action=0`` (training): abort the communicator and exit the process with code 86;
    * ``action=1`` (tests): record the reason; :meth:`check` raises it.

    ``comm_handle=0`` watches the step deadline only."""

    def __init__(self, comm_handle: int, device, timeout_s: float, action: int = 0):
        from ..ops._ext import load_main as load
        self.lib = load()
        dev = torch.device(device)
        self.handle = int(self.lib.rccl_watch_start(int(comm_handle), float(timeout_s),
                                                    int(action), dev.index or 0))
        self.timeout_s = float(timeout_s)

    def mark(self) -> None:
        if self.handle:
            self.lib.rccl_watch_mark(self.handle)

    def status(self) -> str:
        return str(self.lib.rccl_watch_status(self.handle)) if self.handle else ""

    def check(self) -> None:
        why = self.status()
        if why:
            raise RuntimeError(f"communicator watchdog: {why}")

    def close(self) -> None:
        if self.handle:
            self.lib.rccl_watch_stop(self.handle)
            self.handle = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def comm_timeout() -> float:
    """Seconds a step may take before the watchdog declares the job hung
    (``LWAAAI_COMM_TIMEOUT``, default 600, like c10d's default; 0 disables it)."""
    return float(os.environ.get("LWAAAI_COMM_TIMEOUT", "600"))


_NATIVE = {}


def native_rccl(group=None, device=None) -> Optional[NativeRccl]:
    """The process group's native RCCL communicator (created on first use; a collective call, so
    every rank must reach it), or None when the group is not ``nccl`` / ``LWAAAI_NATIVE_RCCL=0``."""
    if not is_dist() or dist.get_backend(group) != "nccl" or \
            os.environ.get("LWAAAI_NATIVE_RCCL", "1") == "0":
        return None
    key = id(group) if group is not None else None
    if key not in _NATIVE:
        _NATIVE[key] = _init_native_agreed(group, device)
    return _NATIVE[key]


def init_timeout() -> float:
    """Deadline (s) on ``ncclCommInitRank`` (``LWAAAI_RCCL_INIT_TIMEOUT``, default 300; 0 = the
    blocking init with no deadline)."""
    return float(os.environ.get("LWAAAI_RCCL_INIT_TIMEOUT", "300"))


def _init_native_agreed(group, device) -> Optional[NativeRccl]:
    """Create the native communicator as one collective decision.

    1. Every rank checks that it can (extension loaded, unique id obtained) and the ranks agree
       (an all-reduce over the c10d group); on a no, nobody enters the RCCL init.
    2. Every rank enters ``ncclCommInitRank``, run on a helper thread that this rank waits for
       against a deadline (``LWAAAI_RCCL_INIT_TIMEOUT``, ``csrc/rccl.cpp rccl_init``; the
       communicator itself is an ordinary blocking one, so no collective can return
       ``ncclInProgress`` inside a captured step), then
       validates it with a probe all-reduce. A rank that raises anywhere in this block — before
       it reached the init, inside it, or at the probe — goes straight to step 3. Its peers are
       then waiting inside an init (or a probe on a half-built communicator) that cannot
       complete: the init deadline abandons their init and they raise as well.
    3. The ranks agree again; if any rank has no communicator, every rank closes its own and all
       fall back to the c10d collectives (eager steps at world > 1), instead of some ranks
       waiting in a collective the others never join.

    What is not covered: a peer that hangs (rather than raises) after the init succeeded
    everywhere leaves the probe blocked; the step watchdog does not run yet at that point. With
    ``LWAAAI_RCCL_INIT_TIMEOUT=0`` the init is the blocking call and step 2's guarantee only
    holds for failures after every rank has finished it."""
    uid = torch.zeros(128, dtype=torch.uint8)
    try:
        from ..ops._ext import load_main as load
        lib = load()
        if rank(group) == 0:
            uid = lib.rccl_unique_id()
        ready = True
    except Exception as e:                     # noqa: BLE001 — reported, then agreed on
        print(f"[lwaaai] native RCCL unavailable on rank {rank(group)}: {e}", flush=True)
        ready = False
    if not agree(ready, group, device):
        print("[lwaaai] native RCCL disabled (not every rank can create it): c10d collectives",
              flush=True)
        return None
    dev = torch.device(device) if device is not None else \
        torch.device("cuda", torch.cuda.current_device())
    uid = _bcast_uid(uid, group, dev)
    comm, err = None, None
    try:
        comm = NativeRccl(group, device, uid=uid)
        # validate the new communicator with one tiny all-reduce before trusting it
        probe = torch.ones(1, dtype=torch.float32, device=dev)
        comm.all_reduce(probe)
        if int(probe.item()) != comm.world:
            raise RuntimeError(f"probe all-reduce gave {probe.item()}, expected {comm.world}")
    except Exception as e:                     # noqa: BLE001
        err = e
        print(f"[lwaaai] native RCCL init failed on rank {rank(group)}: {e}", flush=True)
        if comm is not None:
            comm.close()
            comm = None
    if not agree(comm is not None, group, device):
        if comm is not None:
            comm.close()
        print(f"[lwaaai] native RCCL init failed on some rank ({err or 'peer'}): c10d collectives",
              flush=True)
        return None
    return comm


def shutdown_native() -> None:
    """Close every native communicator (see :meth:`NativeRccl.close`); call before the process
    group is destroyed or the process exits. Captured step graphs holding its collectives are
    released first (``train/graphs.py release_graphs``)."""
    if not _NATIVE:
        return
    import gc
    from ..train.graphs import release_graphs
    release_graphs()
    gc.collect()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    for k in list(_NATIVE):
        c = _NATIVE.pop(k)
        if c is not None:
            c.close()


def all_reduce_max(t: torch.Tensor, group=None) -> torch.Tensor:
    if is_dist() and world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t


def broadcast_coalesced(tensors, src: int = 0, group=None, native: Optional[NativeRccl] = None
                        ) -> None:
    """Broadcast a list of tensors from ``src`` as one flat message per dtype (replaces the private
    ``dist._dist_broadcast_coalesced`` of ``ddp.py:193, 374-377``). ``native``: send GPU tensors
    through that RCCL communicator (stream-ordered, graph-capturable) instead of c10d."""
    if not is_dist() or world_size(group) == 1 or not tensors:
        return
    if native is not None and all(t.is_cuda for t in tensors):
        by_dtype = {}
        for t in tensors:
            by_dtype.setdefault(t.dtype, []).append(t)
        for ts in by_dtype.values():
            if len(ts) == 1 and ts[0].is_contiguous():
                native.broadcast(ts[0].detach(), src)
                continue
            flat = torch.cat([t.detach().reshape(-1) for t in ts])
            native.broadcast(flat, src)
            off = 0
            with torch.no_grad():
                for t in ts:
                    n = t.numel()
                    t.copy_(flat[off:off + n].view_as(t))
                    off += n
        return
    by_dtype = {}
    for t in tensors:
        by_dtype.setdefault((t.dtype, t.device), []).append(t)
    for (_, _), ts in by_dtype.items():
        if len(ts) == 1 and ts[0].is_contiguous():      # already flat: in place, no copies
            dist.broadcast(ts[0].detach(), src=src, group=group)
            continue
        flat = torch.cat([t.detach().reshape(-1) for t in ts])
        dist.broadcast(flat, src=src, group=group)
        off = 0
        with torch.no_grad():
            for t in ts:
                n = t.numel()
                t.copy_(flat[off:off + n].view_as(t))
                off += n


def sum_tensor(tensor: torch.Tensor, group=None) -> torch.Tensor:
    """``dist_utils.sum_tensor`` (dist_utils.py:23-26)."""
    rt = tensor.clone()
    if is_dist():
        dist.all_reduce(rt, op=dist.ReduceOp.SUM, group=group)
    return rt


def reduce_tensor(tensor: torch.Tensor, group=None) -> torch.Tensor:
    return sum_tensor(tensor, group) / world_size(group)


def barrier(group=None, device=None) -> None:
    if is_dist():
        if device is not None and torch.device(device).type == "cuda":
            dist.barrier(group=group, device_ids=[torch.device(device).index or 0])
        else:
            dist.barrier(group=group)
