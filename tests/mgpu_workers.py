"""Rank bodies for ``tests/test_multigpu_gpu.py``: one process per GPU, RCCL ("nccl") process
group, the native communicator (``csrc/rccl.cpp``) and captured steps — the world > 1 default
path. Results travel back as ``(status, value)`` files of plain tensors/lists (our own files)."""
import os
import pickle
import socket
import tempfile
import traceback

import torch
import torch.multiprocessing as mp


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fn, outdir, args, env):
    import datetime

    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), **env)
    if os.environ.get("LWAAAI_TEST_SHARE_GPU") == "1":
        # rehearsal on a one-GPU box: every rank on cuda:0, each rank declared its own "host" so
        # RCCL accepts two ranks on one device (it then moves data over its socket transport)
        os.environ["NCCL_HOSTID"] = f"lwaaai-rank{rank}"
    import faulthandler
    import sys
    faulthandler.enable(file=sys.stderr)          # a rank's fatal signal names its Python frame
    # a rank stuck in a collective prints every thread's stack before the harness gives up on it
    faulthandler.dump_traceback_later(int(os.environ.get("LWAAAI_TEST_STACK_AFTER", "90")),
                                      exit=False, file=sys.stderr)
    res = None
    try:
        from layer_wise_aaai20_amd.parallel.comm import bind_rank_device
        dev = bind_rank_device(rank)
        # every rank a client of the parent's store (run_world): no rank binds the port itself
        store = dist.TCPStore("127.0.0.1", port, world, is_master=False,
                              timeout=datetime.timedelta(seconds=120))
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev, store=store)
        res = ("ok", fn(rank, world, dev, *args))
        faulthandler.cancel_dump_traceback_later()
    except Exception:  # noqa: BLE001
        res = ("err", traceback.format_exc())
    finally:
        with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
            pickle.dump(res, f)
        try:
            from layer_wise_aaai20_amd.parallel import comm
            comm.shutdown_native()
        except Exception:  # noqa: BLE001
            pass
        # the result is on disk: leave without c10d's teardown, whose NCCL communicator
        # finalization waits on the peers
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)


def run_world(fn, world, args=(), env=None):
    """Run ``fn`` on ``world`` spawned ranks. A world that has not finished after
    ``LWAAAI_TEST_WORLD_TIMEOUT`` seconds (default 150; each rank prints every thread's stack at
    ``LWAAAI_TEST_STACK_AFTER``, 90 s) is killed — its own child processes, by PID — and the test
    fails, so a rank stuck in a collective cannot stall the rest of the suite."""
    import datetime
    import time

    import torch.distributed as dist
    limit = float(os.environ.get("LWAAAI_TEST_WORLD_TIMEOUT", "150"))
    # the rendezvous store lives here, on a port the OS picked and this process holds, so no rank
    # races another program for a port found free a moment earlier (a rank then waited in
    # _create_c10d_store until the deadline)
    store = dist.TCPStore("127.0.0.1", 0, world, is_master=True, wait_for_workers=False,
                          timeout=datetime.timedelta(seconds=limit))
    port = store.port
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.start_processes(_worker, args=(world, port, fn, d, args, dict(env or {})),
                                 nprocs=world, start_method="spawn", join=False)
        t0 = time.monotonic()

        def stop(msg):
            for p in ctx.processes:
                if p.is_alive():
                    p.kill()
            for p in ctx.processes:
                p.join(10)
            raise AssertionError(msg)
        while not ctx.join(timeout=5):
            for r in range(world):           # a rank that failed: its peers would wait for it
                f = os.path.join(d, f"r{r}.pkl")
                if os.path.exists(f) and os.path.getsize(f) > 0:
                    try:
                        with open(f, "rb") as fh:
                            status, val = pickle.load(fh)   # written by _worker above
                    except Exception:  # noqa: BLE001  (still being written)
                        continue
                    if status != "ok":
                        stop(f"rank {r} failed:\n{val}")
            if time.monotonic() - t0 > limit:
                stop(f"the {world} ranks did not finish within {limit:.0f} s "
                     "(their stacks are in the captured stderr)")
        out = []
        for r in range(world):
            with open(os.path.join(d, f"r{r}.pkl"), "rb") as f:
                status, val = pickle.load(f)         # written by _worker above
            if status != "ok":
                raise AssertionError(f"rank {r} failed:\n{val}")
            out.append(val)
    del store
    return out


# ----------------------------------------------------------------------------------- bodies
def _gather_cpu(t):
    import torch.distributed as dist
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [p.cpu() for p in parts]


def exchange_vs_oracle(rank, world, dev, mode, method, ef, kw, steps=3):
    """Engine-level: each rank puts a rank-seeded random gradient in its arena and syncs through
    the native communicator; the decoded arena must equal the CPU oracle mean on every rank."""
    from layer_wise_aaai20_amd.compress import reference as ref
    from layer_wise_aaai20_amd.models import resnet as R
    from layer_wise_aaai20_amd.parallel.engine import GradSyncEngine
    torch.manual_seed(0)
    net = R.resnet50().to(dev)
    eng = GradSyncEngine(list(net.named_parameters()), mode=mode, method=method,
                         error_feedback=ef, **kw)
    assert eng._native is not None, "native RCCL communicator not in use"
    sent = {}
    for bi, codec in enumerate(eng.codecs):          # keep each bucket's payload of the step
        orig = codec.compress

        def grab(g, e, step, orig=orig, bi=bi):
            out = orig(g, e, step)
            sent[bi] = out.detach().clone()
            return out
        codec.compress = grab
    errs = []
    for step in range(steps):
        g = torch.Generator(device=dev).manual_seed(1000 * step + rank)
        local = torch.zeros(eng.arena.numel, device=dev)
        for s in eng.arena.segments:
            local[s.offset:s.offset + s.numel] = 1e-2 * torch.randn(s.numel, device=dev,
                                                                    generator=g)
        e_old = eng.ef.clone() if ef else None
        eng.arena.grad.copy_(local)
        eng.sync_now()
        torch.cuda.synchronize(dev)
        got = eng.arena.grad.clone()
        raws = _gather_cpu(local)
        if ef:
            sent_local = local + e_old - eng.ef
            exp = sum(_gather_cpu(sent_local)) / world
            errs.append(float((got.cpu() - exp).abs().max()))
            tol = 1e-5
        elif method in ("RandomDithering", "TernGrad"):
            # every rank's GPU payload, gathered and decoded by the CPU mirror codec: checks the
            # exchange and the rank-ordered dequantise-and-average (encoding: test_kernels_gpu)
            from layer_wise_aaai20_amd.compress.codecs import make_codec
            exp = torch.zeros(eng.arena.numel)
            # the quantised reduce-scatter wire: the all-gather decode of the same codes, rounded
            # to bf16 (the wire's shard all-gather) — bit for bit
            ckw = dict(eng.codec_kw)
            qrs = ckw.get("wire") == "qrs"
            if qrs:
                ckw["wire"] = "sparse"
            for bi, (b, plan) in enumerate(zip(eng.buckets, eng.plans)):
                sl = slice(b.start, b.end)
                pays = _gather_cpu(sent[bi].to(dev))
                cod = make_codec(method, plan, world, rank, **ckw)
                part = torch.zeros(b.end - b.start)
                cod.decompress(pays[rank], torch.cat(pays), part)
                exp[sl] = part.to(torch.bfloat16).float() if qrs else part
            errs.append(float((got.cpu() - exp).abs().max()))
            tol = 1e-6 * float(exp.abs().max())
        elif method in ("Topk", "Thresholdv"):
            # the reference compressor (core.py:175-215) on every rank's raw gradient, averaged
            arg = {"K": kw["K"]} if method == "Topk" else {"V": kw["V"]}
            exp = torch.zeros(eng.arena.numel)
            for r in range(world):
                for s in eng.arena.segments:
                    sl = slice(s.offset, s.offset + s.numel)
                    exp[sl] += ref.compress(raws[r][sl], method, **arg)
            exp /= world
            errs.append(float((got.cpu() - exp).abs().max()))
            tol = 1e-8
        else:
            exp = sum(raws) / world
            errs.append(float((got.cpu() - exp).abs().max()))
            tol = 1e-7
        # identical on every rank, bit for bit
        allg = _gather_cpu(got)
        assert all(torch.equal(allg[0], a) for a in allg[1:]), "decoded gradients differ"
    return errs, tol


def train_graph_vs_eager(rank, world, dev, compress, method, ef, kw, steps=8):
    """Trainer-level: the same per-rank batches through an eager trainer and a HIP-graph trainer
    (collectives captured on the side-stream branches); parameters must be bit-identical across
    ranks and between the two modes."""
    os.environ["LWAAAI_GRAPH_AUTO"] = "0"
    from layer_wise_aaai20_amd.train.imagenet import build_trainer
    out = {}
    for graph in (False, True):
        torch.manual_seed(0)
        tr = build_trainer("resnet50", device=dev, compress=compress, method=method,
                           error_feedback=ef, graph=graph, **kw)
        assert tr.ddp.engine._native is not None
        g = torch.Generator(device=dev).manual_seed(77 + rank)
        losses = []
        for i in range(steps):
            x = torch.randint(0, 256, (8, 64, 64, 3), dtype=torch.uint8, device=dev, generator=g)
            t = torch.randint(0, 1000, (8,), device=dev, generator=g)
            losses.append(float(tr.step(x, t)))
            print(f"[rank {rank}] graph={graph} step {i} loss {losses[-1]:.4f}", flush=True)
        torch.cuda.synchronize(dev)
        p = torch.cat([q.detach().float().reshape(-1) for q in tr.ddp.module.parameters()])
        allp = _gather_cpu(p)
        out[graph] = (p.cpu(), losses, tr.graph_replays,
                      all(torch.equal(allp[0], a) for a in allp[1:]))
        del tr
        torch.cuda.empty_cache()
    return out


def cifar_graph_vs_eager(rank, world, dev, network, compress, method, ef, kw, steps=6):
    """CifarTrainer (BASELINE configs 2 and 3: VGG-16 layer-wise Top-K 0.1 %, AlexNet
    entire-model Top-K + EF) on real RCCL ranks, each rank on its own data order: eager vs
    HIP-graph step, parameters bit-identical across ranks and between the two modes."""
    from layer_wise_aaai20_amd.train.cifar_fast import CifarTrainer
    out = {}
    for graph in (False, True):
        torch.manual_seed(0)
        tr = CifarTrainer(network, device=dev, compress=compress, method=method,
                          error_feedback=ef, batch_size=128, n_train=128 * 8, n_test=128,
                          seed=rank, graph=graph, **kw)
        tr.graphed.auto = False
        tr.graphed.decided = True
        assert tr.ddp.engine._native is not None
        losses = [float(tr.step()) for _ in range(steps)]
        torch.cuda.synchronize(dev)
        p = torch.cat([q.detach().float().reshape(-1) for q in tr.model.parameters()])
        allp = _gather_cpu(p)
        out[graph] = (p.cpu(), losses, tr.graphed.replays,
                      all(torch.equal(allp[0], a) for a in allp[1:]))
        del tr
        torch.cuda.empty_cache()
    return out


def capture_fallback_collective(rank, world, dev):
    """LWAAAI_INJECT_FAULT=capture:1 makes rank 1's capture fail: every rank must then run eagerly
    (no replays anywhere) and the parameters must still agree."""
    os.environ["LWAAAI_GRAPH_AUTO"] = "0"
    from layer_wise_aaai20_amd.train.imagenet import build_trainer
    torch.manual_seed(0)
    tr = build_trainer("resnet50", device=dev, compress="layerwise", method="Topk", K=0.01,
                       graph=True)
    g = torch.Generator(device=dev).manual_seed(5 + rank)
    for _ in range(6):
        x = torch.randint(0, 256, (8, 64, 64, 3), dtype=torch.uint8, device=dev, generator=g)
        t = torch.randint(0, 1000, (8,), device=dev, generator=g)
        tr.step(x, t)
    torch.cuda.synchronize(dev)
    p = torch.cat([q.detach().float().reshape(-1) for q in tr.ddp.module.parameters()])
    allp = _gather_cpu(p)
    return tr.graph_replays, tr.graphed.enabled, all(torch.equal(allp[0], a) for a in allp[1:])


def native_init_fallback(rank, world, dev):
    """LWAAAI_INJECT_FAULT=native_init:1: rank 1 rejects its native communicator; every rank must
    fall back to c10d (no native communicator anywhere) and still train in agreement."""
    from layer_wise_aaai20_amd.train.imagenet import build_trainer
    torch.manual_seed(0)
    tr = build_trainer("resnet50", device=dev, compress="layerwise", method="Topk", K=0.01)
    native = tr.ddp.engine._native is not None
    g = torch.Generator(device=dev).manual_seed(9 + rank)
    for _ in range(3):
        x = torch.randint(0, 256, (8, 64, 64, 3), dtype=torch.uint8, device=dev, generator=g)
        t = torch.randint(0, 1000, (8,), device=dev, generator=g)
        tr.step(x, t)
    torch.cuda.synchronize(dev)
    p = torch.cat([q.detach().float().reshape(-1) for q in tr.ddp.module.parameters()])
    allp = _gather_cpu(p)
    return native, all(torch.equal(allp[0], a) for a in allp[1:])
