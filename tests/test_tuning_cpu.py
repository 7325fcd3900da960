"""Persisted kernel-choice table (``ops/tuning.py``): pinned entries replace timing, and new
decisions are written back so a second process makes the same choices."""
import importlib
import json

import pytest


class _FakeEvent:
    clock = [0.0]

    def __init__(self, enable_timing=True):
        self.t = 0.0

    def record(self):
        self.t = _FakeEvent.clock[0]

    def synchronize(self):
        pass

    def elapsed_time(self, other):
        return other.t - self.t


@pytest.fixture
def tuning(tmp_path, monkeypatch):
    path = tmp_path / "tune.json"
    path.write_text(json.dumps({"gemm|(1, 2, 3)": 22, "linear|('fwd', 8)": [21, 4]}))
    monkeypatch.setenv("LWAAAI_TUNE_FILE", str(path))
    monkeypatch.delenv("RANK", raising=False)
    import layer_wise_aaai20_amd.ops.tuning as T
    T = importlib.reload(T)
    monkeypatch.setattr(T.torch.cuda, "Event", _FakeEvent)
    monkeypatch.setattr(T.torch.cuda, "is_current_stream_capturing", lambda: False)
    yield T, path
    monkeypatch.delenv("LWAAAI_TUNE_FILE")
    importlib.reload(T)


def test_pinned_entries_skip_timing(tuning):
    T, _ = tuning

    def run(c):
        raise AssertionError("a pinned choice must not be timed")
    assert T.Tuner("gemm", "X").pick((1, 2, 3), run, (1, 2, 21, 22), 0) == 22
    assert T.Tuner("linear", "X").pick(("fwd", 8), run, [(1, 1), (21, 4)], (0, 1)) == (21, 4)


def test_new_decision_is_persisted(tuning):
    T, path = tuning
    cost = {1: 5.0, 2: 1.0, 3: 7.0}

    def run(c):                      # each call advances the fake clock by the candidate's cost
        _FakeEvent.clock[0] += cost[c]
    tu = T.Tuner("conv", "X")
    assert tu.pick(("k", 64), run, (1, 2, 3), 1) == 2
    saved = json.loads(path.read_text())
    assert saved["conv|('k', 64)"] == 2
    assert saved["gemm|(1, 2, 3)"] == 22          # existing entries kept
    # a fresh tuner (another process) reads the pinned choice
    T2 = importlib.reload(T)
    assert T2.Tuner("conv", "X").pick(("k", 64), lambda c: 1 / 0, (1, 2, 3), 1) == 2


def test_disabled_uses_default(monkeypatch):
    import layer_wise_aaai20_amd.ops.tuning as T
    monkeypatch.setenv("LWAAAI_X_OFF", "0")
    monkeypatch.setattr(T.torch.cuda, "is_current_stream_capturing", lambda: False)
    assert T.Tuner("q", "LWAAAI_X_OFF").pick(7, lambda c: 1 / 0, (1, 2), 9) == 9


def test_stale_pinned_entry_is_timed(tuning):
    """A pinned choice that is not among the current candidates is ignored (and timed)."""
    T, _ = tuning
    cost = {1: 5.0, 2: 1.0}

    def run(c):
        _FakeEvent.clock[0] += cost[c]
    with pytest.warns(UserWarning, match="stale tuning entry"):
        assert T.Tuner("gemm", "X").pick((1, 2, 3), run, (1, 2), 1) == 2


def test_shipped_table_default_and_none(monkeypatch):
    import layer_wise_aaai20_amd.ops.tuning as T
    monkeypatch.delenv("LWAAAI_TUNE_FILE", raising=False)
    T = importlib.reload(T)
    assert T._READ == T.SHIPPED and T._FILE == ""           # read-only: never written back
    monkeypatch.setenv("LWAAAI_TUNE_FILE", "none")
    T = importlib.reload(T)
    assert T.table() == {} and T._FILE == ""
    monkeypatch.delenv("LWAAAI_TUNE_FILE")
    importlib.reload(T)


def _w_agree_tuner(rank, world):
    import layer_wise_aaai20_amd.ops.tuning as T
    T.torch.cuda.Event = _FakeEvent
    T.torch.cuda.is_current_stream_capturing = lambda: False
    # rank 0 finds candidate 1 fastest, rank 1 finds 3 fastest; summed, 2 wins
    cost = [{1: 1.0, 2: 2.0, 3: 9.0}, {1: 9.0, 2: 2.0, 3: 1.0}][rank]

    def run(c):
        _FakeEvent.clock[0] += cost[c]
    local = T.Tuner("agree-a", "X").pick(("k",), run, (1, 2, 3), 1)
    with T.rank_agreement():
        agreed = T.Tuner("agree-b", "X").pick(("k",), run, (1, 2, 3), 1)
    return local, agreed


def test_rank_agreement_picks_one_kernel_for_all_ranks():
    from dist_utils import run_world
    (l0, a0), (l1, a1) = run_world(_w_agree_tuner, 2)
    assert (l0, l1) == (1, 3)          # timed alone, the ranks disagree
    assert a0 == a1 == 2               # agreed: the candidate with the lowest summed time
