"""The 32x32x16-MFMA twins of the tiled GEMM (csrc/gemm_core.h k_gemm MF = 32, GemmTile ids
41..46 = tiles 1..6 + 40) against fp32 torch: every tile x operand layout x split-K, the bf16
epilogues (column statistics, prologue, ReLU-masked addend, backward BN statistics) and the
implicit-GEMM convolutions (forward with BN prologue + statistics, data gradient incl. stride-2
parity classes, weight gradient) on the same kernels. The MF = 32 accumulator holds four runs of
4 columns per lane and its statistics fold over a 32-lane half-wave, so each of those paths is
checked here on ragged shapes."""
import pytest
import torch
import torch.nn.functional as F

from layer_wise_aaai20_amd.ops import conv as CV
from layer_wise_aaai20_amd.ops import gemm as G

pytestmark = pytest.mark.gpu

MF32 = [41, 42, 43, 44, 45, 46]
DIMS = {41: (128, 128, 32), 42: (128, 128, 64), 43: (256, 64, 32), 44: (64, 256, 32),
        45: (256, 64, 64), 46: (64, 64, 64)}


def _lib():
    return G.load()


@pytest.mark.parametrize("tile", MF32)
@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K", [(520, 200, 328), (64, 64, 64), (1000, 136, 72)])
def test_mf32_tiles_fp32_out(tile, a_kc, b_kc, M, N, K):
    torch.manual_seed(tile + M)
    if not a_kc and M % 8:
        pytest.skip("M-contiguous A needs M % 8 == 0")
    if not b_kc and N % 8:
        pytest.skip("N-contiguous B needs N % 8 == 0")
    Am = torch.randn(M, K, device="cuda").bfloat16()
    Bm = torch.randn(K, N, device="cuda").bfloat16()
    A = Am.contiguous() if a_kc else Am.t().contiguous()
    B = Bm.t().contiguous() if b_kc else Bm.contiguous()
    ref = Am.float() @ Bm.float()
    for splits in (1, 3):
        C, _ = G.gemm_ex(A, K if a_kc else M, a_kc, B, K if b_kc else N, b_kc, M, N, K,
                         splits=splits, out_bf16=False, tile=tile)
        torch.testing.assert_close(C, ref, rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("tile", MF32)
def test_mf32_bias_relu_and_stats(tile):
    lib = _lib()
    torch.manual_seed(tile)
    M, N, K = 1000, 136, 96
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    C, st = G.gemm_ex(x, K, True, w, K, True, M, N, K, tile=tile, stats=True)
    ref = x.float() @ w.float().t()
    torch.testing.assert_close(C.float(), ref, rtol=2e-2, atol=5e-2)
    bm = DIMS[tile][0]
    assert st.shape == (-(-M // bm), 2, N)
    c = C.float()
    torch.testing.assert_close(st[:, 0].sum(0), c.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(st[:, 1].sum(0), (c * c).sum(0), rtol=1e-4, atol=1e-1)
    torch.testing.assert_close(st[0, 0], c[:bm].sum(0), rtol=1e-4, atol=1e-2)
    b = torch.randn(N, device="cuda")
    y = lib.gemm_ex(x, K, True, w, K, True, M, N, K, b, True, 1, True, tile, None, None, True,
                    False)[0]
    torch.testing.assert_close(y.float(), torch.relu(ref + b), rtol=2e-2, atol=5e-2)


@pytest.mark.parametrize("tile", MF32)
def test_mf32_prologues(tile):
    torch.manual_seed(3 + tile)
    M, N, K = 704, 192, 136
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    sc = torch.rand(K, device="cuda") + 0.5
    sh = torch.randn(K, device="cuda")
    # the prologue is one fmaf per element (x*sc exact in double, one rounding to fp32)
    a = torch.relu((x.double() * sc.double() + sh.double()).float()).bfloat16().float()
    y, _ = G.gemm_ex(x, K, True, w, K, True, M, N, K, out_bf16=False, pro_scale=sc, pro_shift=sh,
                     pro_on_a=True, tile=tile)
    torch.testing.assert_close(y, a @ w.float().t(), rtol=1e-3, atol=1e-2)
    dy = torch.randn(M, N, device="cuda").bfloat16()
    dw, _ = G.gemm_ex(dy, N, False, x, K, False, N, K, M, splits=3, out_bf16=False, pro_scale=sc,
                      pro_shift=sh, pro_on_a=False, tile=tile)
    torch.testing.assert_close(dw, dy.float().t() @ a, rtol=1e-3, atol=5e-2)


def _bits_of(keep):
    return (keep.view(-1, 8).to(torch.uint8) <<
            torch.arange(8, device="cuda", dtype=torch.uint8)).sum(1).to(torch.uint8)


@pytest.mark.parametrize("tile", MF32)
def test_mf32_masked_addend(tile):
    """dy·W + dres·[bit] rounded as the MF = 16 twin rounds it."""
    lib = _lib()
    torch.manual_seed(6 + tile)
    M, N, K = 1000, 96, 128
    A = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
    B = (torch.randn(K, N, device="cuda") * 0.5).bfloat16()
    add = torch.randn(M, N, device="cuda").bfloat16()
    keep = torch.rand(M, N, device="cuda") > 0.4
    add_bits = _bits_of(keep)
    C, _ = lib.gemm_ex(A, K, True, B, N, False, M, N, K, None, False, 1, True, tile, None, None,
                       True, False, None, add, False, 0, add_bits)
    base = (A.float() @ B.float()).bfloat16().float()
    ref = (base + add.float() * keep).bfloat16().float()
    torch.testing.assert_close(C.float(), ref, atol=3e-2, rtol=2e-2)


def _pin(monkeypatch, choice):
    monkeypatch.setattr(CV.TUNER, "pick", lambda key, run, cands, default, c=choice: c)


@pytest.mark.parametrize("shape", [(4, 64, 14, 14, 64), (3, 128, 9, 11, 96)])
@pytest.mark.parametrize("tile", [41, 42, 43, 45, 46])
def test_mf32_conv_fwd_with_bn_prologue_and_stats(shape, tile, monkeypatch):
    n, c, h, w, co = shape
    torch.manual_seed(tile)
    x = torch.randn(n, c, h, w, device="cuda").bfloat16().contiguous(
        memory_format=torch.channels_last)
    wt = (torch.randn(co, c, 3, 3, device="cuda") * 0.1).bfloat16().contiguous(
        memory_format=torch.channels_last)
    sc = torch.rand(c, device="cuda") + 0.5
    sh = torch.randn(c, device="cuda") * 0.1
    _pin(monkeypatch, tile)
    y, st = CV.conv_fwd(x, wt, 1, 1, pro=(sc, sh), stats=True)
    a = torch.relu((x.double() * sc.double().view(1, -1, 1, 1) +
                    sh.double().view(1, -1, 1, 1)).float()).bfloat16().float()
    ref = F.conv2d(a, wt.float(), None, 1, 1)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=5e-2)
    yr = y.float().permute(0, 2, 3, 1).reshape(-1, co)
    torch.testing.assert_close(st[:, 0].sum(0), yr.sum(0), rtol=1e-3, atol=5e-2)


@pytest.mark.parametrize("stride", [1, 2])
@pytest.mark.parametrize("tile", [41, 42, 43, 45, 46])
def test_mf32_conv_dgrad(stride, tile, monkeypatch):
    torch.manual_seed(tile + stride)
    n, c, h, co = 3, 64, 12, 96
    x = torch.randn(n, c, h, h, device="cuda").bfloat16().float().requires_grad_()
    wt = (torch.randn(co, c, 3, 3, device="cuda") * 0.1).bfloat16()
    y = F.conv2d(x, wt.float(), None, stride, 1)
    dy = torch.randn_like(y).bfloat16()
    y.backward(dy.float())
    dyc = dy.contiguous(memory_format=torch.channels_last)
    w2 = wt.contiguous(memory_format=torch.channels_last)
    for layout in ("nkc", "kc"):
        _pin(monkeypatch, (layout, tile))
        dx = CV.conv_dgrad(dyc, w2, (h, h), stride, 1)
        torch.testing.assert_close(dx.float(), x.grad, rtol=2e-2, atol=5e-2)


@pytest.mark.parametrize("tile", [41, 42, 44, 46])
def test_mf32_conv_wgrad(tile, monkeypatch):
    torch.manual_seed(tile)
    n, c, h, co = 4, 64, 14, 128
    x = torch.randn(n, c, h, h, device="cuda").bfloat16()
    wt = torch.randn(co, c, 3, 3, device="cuda").float().requires_grad_()
    y = F.conv2d(x.float(), wt, None, 1, 1)
    dy = torch.randn_like(y).bfloat16()
    y.backward(dy.float())
    _pin(monkeypatch, (tile, 4))
    dw = CV.conv_wgrad(dy.contiguous(memory_format=torch.channels_last),
                       x.contiguous(memory_format=torch.channels_last), (co, c, 3, 3), 1, 1)
    torch.testing.assert_close(dw.float(), wt.grad, rtol=2e-2, atol=2e-1)


def test_mf32_twins_are_tuner_candidates():
    from layer_wise_aaai20_amd.ops import block as BK
    from layer_wise_aaai20_amd.ops.tuning import MF32_ON
    if not MF32_ON:
        pytest.skip("32x32 twins disabled")
    assert set(MF32) <= set(BK.TILES)
    assert {41, 42, 43, 45, 46} <= set(CV.ROW_TILES) and {41, 42, 44, 46} <= set(CV.COL_TILES)
