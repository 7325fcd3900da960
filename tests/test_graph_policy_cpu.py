"""Which compressors the whole-step HIP graph may capture (train/graphs.py): the decision is
made from codec flags on the host, so it is checked here without a GPU."""
import numpy as np
import torch

from layer_wise_aaai20_amd.compress import codecs as C
from layer_wise_aaai20_amd.compress.plan import SegPlan
from layer_wise_aaai20_amd.parallel.engine import GradSyncEngine
from layer_wise_aaai20_amd.train.graphs import StepGraph


def _plan():
    return SegPlan([0, 4096], [4096, 20000])


def test_codec_graph_flags():
    p = _plan()
    mk = lambda m, **kw: C.make_codec(m, p, 2, 0, seed=1, **kw)  # noqa: E731
    assert mk("Topk", K=0.01).graph_safe
    assert mk("none").graph_safe
    assert mk("TernGrad").graph_safe
    assert mk("RandomDithering", qstates=255).graph_safe
    assert mk("Randomk", K=0.05).graph_safe           # device step counter keys masks
    assert mk("Thresholdv", V=1e-3, wire="sparse-capped").graph_safe   # fixed capacity
    assert not mk("Thresholdv", V=1e-3, wire="sparse").graph_safe   # host read of capacity
    assert not mk("Thresholdv", V=1e-3, wire="sparse-exact").graph_safe
    assert mk("AdaptiveThreshold", wire="sparse-capped").graph_safe
    assert mk("Thresholdv", V=1e-3).graph_safe                      # default dense wire
    assert mk("Topk", K=0.5, wire="dense").graph_safe


def test_engine_and_stepgraph_are_eager_on_cpu():
    params = [("w", torch.nn.Parameter(torch.randn(64, 64)))]
    eng = GradSyncEngine(params, mode="layerwise", method="Topk", K=0.01, world_size=1)
    assert not eng.graph_safe()                   # CPU arena: nothing to capture
    calls = []
    sg = StepGraph(lambda x: calls.append(x) or x * 2, eng, object(), "cpu")
    assert not sg.enabled
    x = torch.ones(3)
    assert torch.equal(sg(x), x * 2) and len(calls) == 1 and sg.replays == 0


def test_device_step_counter_absent_on_cpu():
    params = [("w", torch.nn.Parameter(torch.randn(128)))]
    eng = GradSyncEngine(params, mode="entiremodel", method="RandomDithering", qstates=255,
                         world_size=1)
    assert eng._dstep is None and all(c.step_t is None for c in eng.codecs)
    eng.set_step(7)
    assert eng.step == 7
    assert np.isfinite(eng.step)
