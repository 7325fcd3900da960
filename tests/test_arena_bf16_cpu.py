"""Per-forward bf16 weight mirror of the flat parameter arena (parallel/arena.py): views are handed
out only while neither the flat buffer nor the parameter changed since the refresh."""
import torch

from layer_wise_aaai20_amd.ops.block import _bf16_weight
from layer_wise_aaai20_amd.parallel.arena import GradArena


def test_mirror_tracks_versions():
    m = torch.nn.Conv2d(8, 16, 1, bias=False)
    a = GradArena(list(m.named_parameters()), flat_params=True)
    assert getattr(m.weight, "_lw_bf16_of", None) is None  # never refreshed
    a.refresh_bf16()
    v = m.weight._lw_bf16_of()
    assert v is not None and v.dtype == torch.bfloat16 and v.shape == m.weight.shape
    assert torch.equal(v.float(), m.weight.detach().bfloat16().float())
    assert _bf16_weight(m.weight).data_ptr() == v.data_ptr()
    with torch.no_grad():
        m.weight.mul_(2)                                # in-place on the parameter
    assert m.weight._lw_bf16_of() is None
    w = _bf16_weight(m.weight)                          # falls back to a cast
    assert torch.equal(w.float(), m.weight.detach().bfloat16().float())
    a.refresh_bf16()
    assert m.weight._lw_bf16_of() is not None
    a.param_buf.add_(1.0)                               # optimizer-style write via the buffer
    assert m.weight._lw_bf16_of() is None
    m.load_state_dict(m.state_dict())
    a.refresh_bf16()
    assert m.weight._lw_bf16_of() is not None
