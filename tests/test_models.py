"""Model definitions match the reference's parameter inventory."""
import pytest
import torch

from layer_wise_aaai20_amd.models import cifar, resnet
from layer_wise_aaai20_amd.models.graph import build_graph, rel_path, union, Identity, Add


def count(m):
    ps = [p for p in m.parameters() if p.requires_grad]
    return len(ps), sum(p.numel() for p in ps), max(p.numel() for p in ps)


@pytest.mark.parametrize("name,tensors,params,largest", [
    ("Resent9", 25, 6_573_120, 2_359_296),
    ("Alexnet", 16, 2_255_296, 884_736),
    ("Alexnet1", 16, 23_272_266, 16_777_216),
])
def test_cifar_inventory(name, tensors, params, largest):
    assert count(cifar.build_network(name)) == (tensors, params, largest)


def test_vgg16_inventory():
    m = cifar.vgg16()
    assert count(m) == (32, 134_301_514, 102_760_448)
    out = m({"input": torch.randn(2, 3, 32, 32), "target": torch.tensor([1, 2])})
    assert out["loss"].shape == (2,) and out["correct"].dtype == torch.bool


def test_resnet50_inventory_and_names():
    m = resnet.resnet50()
    assert count(m) == (161, 25_557_032, 2_359_296)
    sizes = [p.numel() for p in m.parameters()]
    assert sum(1 for s in sizes if s <= 4096) == 108
    keys = list(m.state_dict())
    assert "layer1.0.downsample.1.running_mean" in keys and "fc.bias" in keys
    assert len(keys) == 320


def test_resnet9_forward_dict_and_message_order():
    m = cifar.build_network("resnet9")
    out = m({"input": torch.randn(4, 3, 32, 32), "target": torch.randint(0, 10, (4,))})
    assert out["loss"].shape == (4,) and "classifier" in out
    sizes = [p.numel() for p in m.parameters()]
    assert sizes[:4] == [1728, 64, 64, 73728] and sizes[-1] == 5120


def test_bn0_init():
    m = resnet.resnet50(bn0=True)
    assert float(m.layer1[0].bn3.weight.abs().sum()) == 0.0


def test_build_graph_relative_inputs():
    net = {"a": Identity(), "blk": {"in": Identity(), "x": Identity(),
                                    "add": (Add(), [rel_path("in"), rel_path("x")])}}
    g = build_graph(net)
    assert g["a"][1] == ["input"] and g["blk_in"][1] == ["a"]
    assert g["blk_add"][1] == ["blk_in", "blk_x"]
