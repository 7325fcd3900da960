"""StepGraph bookkeeping without a GPU: one captured graph per input signature, per-signature
eager warm-up (an epoch's odd-sized last batch neither evicts the full-size graph nor is captured
on first sight), LRU bound, and the graph-vs-eager decision that discards the first replay and
compares averages. Capture and replay are replaced by a fake that re-runs the step closure."""
import types

import torch

from layer_wise_aaai20_amd.train.graphs import StepGraph


class _Opt:
    device_hyper = False

    def graph_signature(self):
        return ("sgd",)

    def load_hyper(self):
        pass


class _Eng:
    world = 1
    step = 0

    def __init__(self):
        self.stats = types.SimpleNamespace(steps=0)

    def graph_safe(self):
        return True

    def _reset_state(self):
        pass


class FakeStepGraph(StepGraph):
    def __init__(self, fn, eager_ms, graph_ms, **kw):
        super().__init__(fn, _Eng(), _Opt(), "cpu", **kw)
        self.enabled = True
        self.kinds = []
        self._clock = {"eager": eager_ms, "graph": graph_ms}
        self._now = None

    def _capture(self, inputs, sig):
        static_in = [t.clone() for t in inputs]
        out = {}
        sg = self

        class G:
            def replay(self_):
                sg.kinds.append("replay")
                out["y"] = sg.fn(*static_in)

        g = (G(), static_in, out)
        while len(self._graphs) >= self.MAX_GRAPHS:
            self._graphs.pop(next(iter(self._graphs)))
        self._graphs[sig] = g
        self.captures += 1
        self.kinds.append("capture")
        return g

    def _mark(self):
        self._now = len(self.kinds)

    def _lap(self):
        kind = "graph" if self.kinds and self.kinds[-1] == "replay" else "eager"
        return self._clock[kind]


def _fn(log):
    def fn(x):
        log.append(tuple(x.shape))
        return x * 2
    return fn


def test_per_signature_graphs_and_warmup():
    log = []
    sg = FakeStepGraph(_fn(log), eager_ms=10.0, graph_ms=5.0, warmup=2, auto=False)
    full, odd = torch.ones(4, 3), torch.ones(2, 3)
    for _ in range(2):
        sg(full)                       # eager warm-up of the full-size signature
    assert sg.captures == 0 and sg.replays == 0
    sg(full)                           # capture + replay
    assert sg.captures == 1 and sg.replays == 1
    sg(odd)                            # new signature: eager, full-size graph kept
    assert sg.captures == 1 and len(sg._graphs) == 1
    sg(full)
    assert sg.replays == 2 and sg.captures == 1
    sg(odd)                            # second sight: still warming up (warmup=2)
    sg(odd)                            # third: captured
    assert sg.captures == 2 and len(sg._graphs) == 2
    sg(full)
    assert sg.captures == 2 and sg.replays == 4
    assert sg.engine.step == 4         # host mirror of the device step counter per replay


def test_lru_bound():
    sg = FakeStepGraph(_fn([]), 1.0, 1.0, warmup=0, auto=False)
    for n in range(1, StepGraph.MAX_GRAPHS + 3):
        sg(torch.ones(n))
    assert len(sg._graphs) == StepGraph.MAX_GRAPHS


def test_decision_keeps_faster_graph_and_discards_first_replay():
    sg = FakeStepGraph(_fn([]), eager_ms=10.0, graph_ms=5.0, warmup=4, auto=True, timed=3)
    x = torch.ones(3)
    for _ in range(4 + 1 + 3):         # warm-up, upload replay, timed replays
        sg(x)
    assert sg.decided and sg.enabled and sg.choice == (5.0, 10.0)
    assert len(sg._replay_t) == 4      # first replay recorded but excluded from the mean


def test_decision_drops_slower_graph():
    calls = []
    sg = FakeStepGraph(_fn(calls), eager_ms=5.0, graph_ms=6.0, warmup=3, auto=True, timed=2)
    x = torch.ones(3)
    for _ in range(3 + 1 + 2):
        sg(x)
    assert sg.decided and not sg.enabled and not sg._graphs
    n, r = len(calls), sg.replays
    sg(x)                              # eager from now on
    assert len(calls) == n + 1 and sg.replays == r
