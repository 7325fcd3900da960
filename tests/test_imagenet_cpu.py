"""ImageNet training machinery on CPU: schedules, LR scheduler, data phases, checkpoint/resume,
metrics helpers, synthetic data pipeline."""
import os

import pytest
import torch

from layer_wise_aaai20_amd.data import imagenet as D
from layer_wise_aaai20_amd.train import imagenet_main as T
from layer_wise_aaai20_amd.train.schedules import schedule, schedules


class _Opt:
    def __init__(self):
        self.param_groups = [{"lr": 0.0}, {"lr": 0.0}]


def test_schedules_inventory():
    assert set(schedules) == {1, 2, 4, 8, 16}
    one = schedule("one_machine")
    assert one[0] == {"ep": 0, "sz": 128, "bs": 512, "trndir": "-sz/160"}
    assert max(max(T.listify(p["ep"])) for p in one if "lr" in p) == 35


def test_scheduler_warmup_and_steps():
    ph = [p for p in schedule(1) if "lr" in p]
    s = T.Scheduler(_Opt(), ph)
    assert s.tot_epochs == 35
    assert s.get_lr(0, 0, 100) == pytest.approx(1.0)
    assert s.get_lr(2, 50, 100) == pytest.approx(1.0 + 2.5 / 5)     # linear 1.0 -> 2.0 over ep 0-5
    assert s.get_lr(10, 3, 100) == pytest.approx(1.0)
    assert s.get_lr(15, 0, 100) == pytest.approx(224 / 512)
    assert s.get_lr(34, 0, 100) == pytest.approx(1.0 / 1000 * 128 / 512)
    s.update_lr(15, 1, 100)
    assert all(g["lr"] == pytest.approx(224 / 512) for g in s.optimizer.param_groups)


def test_listify_and_correct():
    assert T.listify(3) == [3] and T.listify((1, 2)) == [1, 2] and T.listify(5, [1, 2]) == [5, 5]
    out = torch.tensor([[0.1, 0.9, 0.0], [0.8, 0.1, 0.1]])
    c1, c2 = T.correct(out, torch.tensor([1, 2]), topk=(1, 2))
    assert float(c1) == 1 and float(c2) == 1
    a1, = T.accuracy(out, torch.tensor([1, 0]), topk=(1,))
    assert float(a1) == 100.0


def test_dist_val_sampler_and_rect_shapes():
    s0 = D.DistValSampler(list(range(10)), 3, distributed=False, rank=0, world=2)
    s1 = D.DistValSampler(list(range(10)), 3, distributed=False, rank=1, world=2)
    assert [len(b) for b in s0] == [3, 3] and [len(b) for b in s1] == [3, 1]
    ar = D.sort_ar(16)
    idx2ar = D.map_idx2ar(ar, 4)
    ds = D.RectValDataset(D.SyntheticImageNet(16, 32), idx2ar, 32)
    order = [i for _, i in ar]
    shapes = {ds[i][0].shape for i in order[:4]}
    assert len(shapes) == 1                                   # one shape per batch
    h, w, c = shapes.pop()
    assert c == 3 and min(h, w) == 32 and h % 8 == 0 and w % 8 == 0


def test_get_loaders_synthetic_cpu():
    trn, val, tsmp, vsmp = D.get_loaders(sz=32, bs=8, val_bs=8, n_train=32, n_val=16,
                                         device="cpu")
    x, y = next(iter(trn))
    assert x.shape == (8, 3, 32, 32) and x.dtype == torch.float32 and y.shape == (8,)
    assert x.is_contiguous(memory_format=torch.channels_last)
    assert abs(float(x.mean())) < 0.5


def test_train_resume_checkpoint_layout(tmp_path):
    logdir = str(tmp_path / "run")
    args = ["synthetic", "--phases", "smoke", "--short-epoch", "--arch", "resnet18", "--logdir",
            logdir, "-c", "layerwise", "--method", "Topk", "-K", "0.01", "--epochs", "1",
            "--print-freq", "100", "--device", "cpu", "--extra-ckpt"]
    T.main(args)
    ck = torch.load(os.path.join(logdir, "checkpoint.pth.tar"), weights_only=True)
    assert {"epoch", "state_dict", "best_top5", "optimizer"} <= set(ck)
    assert ck["epoch"] == 1 and "scheduler" in ck
    assert "fc.weight" in ck["state_dict"]
    ev = open(os.path.join(logdir, "event.log")).read()
    assert "~~epoch\thours\ttop1\ttop5" in ev and "~~0\t" in ev
    # resume continues at epoch 1 and writes epoch 2
    T.main(args + ["--resume", os.path.join(logdir, "checkpoint.pth.tar")])
    ck2 = torch.load(os.path.join(logdir, "checkpoint.pth.tar"), weights_only=True)
    assert ck2["epoch"] == 2


@pytest.mark.parametrize("compress,method", [("enitremodel", "Topk"), ("none", "none")])
def test_train_modes_run(tmp_path, compress, method):
    T.main(["synthetic", "--phases", "smoke", "--short-epoch", "--arch", "resnet18",
            "--logdir", str(tmp_path), "-c", compress, "--method", method, "-K", "0.01",
            "--epochs", "1", "--device", "cpu", "--print-freq", "100"])


def test_adapt_state_dict_prefix():
    import torch
    from layer_wise_aaai20_amd.train.imagenet_main import adapt_state_dict
    m = torch.nn.Linear(2, 2)
    wrapped = torch.nn.Module()
    wrapped.module = torch.nn.Linear(2, 2)
    sd_wrapped = wrapped.state_dict()
    assert set(adapt_state_dict(sd_wrapped, m)) == set(m.state_dict())
    assert set(adapt_state_dict(m.state_dict(), wrapped)) == set(sd_wrapped)
    m.load_state_dict(adapt_state_dict(sd_wrapped, m))
