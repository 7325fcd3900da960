"""Hand-written MFMA GEMM vs fp32 torch matmul (all four operand layouts, bias/ReLU epilogue,
split-K, ragged edges) and the MFMALinear layer vs nn.Linear."""
import pytest
import torch

from layer_wise_aaai20_amd.ops import gemm as G

pytestmark = pytest.mark.gpu


def _ref(A, B):
    return A.float() @ B.float()


def _lib():
    from layer_wise_aaai20_amd.ops._ext import load
    return load()


@pytest.mark.parametrize("M,N,K", [(128, 128, 32), (256, 384, 512), (200, 136, 72),
                                   (1000, 64, 2048), (64, 1000, 136), (8, 16, 8)])
@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("splits", [1, 3])
def test_gemm_layouts(M, N, K, a_kc, b_kc, splits):
    torch.manual_seed(0)
    if not a_kc and M % 8:
        pytest.skip("M-contiguous A needs M % 8 == 0")
    if not b_kc and N % 8:
        pytest.skip("N-contiguous B needs N % 8 == 0")
    Am = torch.randn(M, K, device="cuda").bfloat16()      # logical A[m][k]
    Bm = torch.randn(K, N, device="cuda").bfloat16()      # logical B[k][n]
    A = Am.contiguous() if a_kc else Am.t().contiguous()  # stored [M][K] or [K][M]
    B = Bm.t().contiguous() if b_kc else Bm.contiguous()  # stored [N][K] or [K][N]
    lda = K if a_kc else M
    ldb = K if b_kc else N
    C = G.gemm(A, lda, a_kc, B, ldb, b_kc, M, N, K, None, False, splits, False)
    torch.testing.assert_close(C, _ref(Am, Bm), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("relu", [False, True])
def test_gemm_bias_relu_bf16_out(relu):
    M, N, K = 300, 264, 96
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    b = torch.randn(N, device="cuda")
    y = G.linear_fwd(x, w, b, relu)
    r = x.float() @ w.float().t() + b
    r = torch.relu(r) if relu else r
    torch.testing.assert_close(y.float(), r, rtol=2e-2, atol=5e-2)


def test_mfma_linear_matches_nn_linear():
    torch.manual_seed(0)
    lin = torch.nn.Linear(256, 136).cuda()
    ref = torch.nn.Linear(256, 136).cuda()
    ref.load_state_dict(lin.state_dict())
    with torch.no_grad():                       # same bf16-rounded operands on both sides
        ref.weight.copy_(ref.weight.bfloat16().float())
    G.to_mfma_linear(lin, fuse_relu=False)
    x = torch.randn(64, 256, device="cuda", requires_grad=True)
    xr = x.detach().clone().requires_grad_()
    y = lin(x)
    yr = ref(xr.bfloat16().float())
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=5e-2)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    torch.testing.assert_close(lin.weight.grad, ref.weight.grad, rtol=3e-2, atol=1e-1)
    torch.testing.assert_close(lin.bias.grad, ref.bias.grad, rtol=3e-2, atol=1e-1)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=3e-2, atol=5e-2)


@pytest.mark.parametrize("tile", ["128x128x32", "128x128x64", "256x64x32", "64x256x32",
                                  "256x64x64", "64x64x64"])
@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, True), (False, False)])
def test_gemm_tiles(tile, a_kc, b_kc):
    torch.manual_seed(1)
    M, N, K = 520, 200, 328
    Am = torch.randn(M, K, device="cuda").bfloat16()
    Bm = torch.randn(K, N, device="cuda").bfloat16()
    A = Am.contiguous() if a_kc else Am.t().contiguous()
    B = Bm.t().contiguous() if b_kc else Bm.contiguous()
    for splits in (1, 2):
        C, _ = G.gemm_ex(A, K if a_kc else M, a_kc, B, K if b_kc else N, b_kc, M, N, K,
                         splits=splits, out_bf16=False, tile=tile)
        torch.testing.assert_close(C, _ref(Am, Bm), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("tile", ["128x128x32", "256x64x32", "64x256x32", "64x64x64",
                                  "256x256x64", "256x128x64"])
def test_gemm_stats_epilogue(tile):
    """Per-column Σ / Σ² of the bf16 output per M-tile (BatchNorm statistics in the epilogue)."""
    torch.manual_seed(2)
    M, N, K = 1000, 136, 96
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    C, st = G.gemm_ex(x, K, True, w, K, True, M, N, K, tile=tile, stats=True)
    bm = {"128x128x32": 128, "256x64x32": 256, "64x256x32": 64, "64x64x64": 64,
          "256x256x64": 128, "256x128x64": 128}[tile]   # big tiles: one row per wave row
    tiles_m = -(-M // bm)
    assert st.shape == (tiles_m, 2, N)
    c = C.float()
    torch.testing.assert_close(st[:, 0].sum(0), c.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(st[:, 1].sum(0), (c * c).sum(0), rtol=1e-4, atol=1e-1)
    # per-tile partials
    torch.testing.assert_close(st[0, 0], c[:bm].sum(0), rtol=1e-4, atol=1e-2)


def test_gemm_prologue_a_and_b():
    """relu(v*scale+shift) applied while loading: per-k on a K-contiguous A (forward of a 1x1 conv
    on a BatchNorm'd input) and per-n on an N-contiguous B (its weight gradient)."""
    torch.manual_seed(3)
    M, N, K = 704, 192, 136
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    sc = torch.rand(K, device="cuda") + 0.5
    sh = torch.randn(K, device="cuda")
    a = torch.relu(x.float() * sc + sh).bfloat16().float()
    y, _ = G.gemm_ex(x, K, True, w, K, True, M, N, K, out_bf16=False, pro_scale=sc, pro_shift=sh,
                     pro_on_a=True)
    torch.testing.assert_close(y, a @ w.float().t(), rtol=1e-3, atol=1e-2)
    # weight gradient: dW[N][K] = dyᵀ · a, B = x (N-contiguous over K channels), prologue per-n
    dy = torch.randn(M, N, device="cuda").bfloat16()
    dw, _ = G.gemm_ex(dy, N, False, x, K, False, N, K, M, splits=3, out_bf16=False, pro_scale=sc,
                      pro_shift=sh, pro_on_a=False)
    torch.testing.assert_close(dw, dy.float().t() @ a, rtol=1e-3, atol=5e-2)


@pytest.mark.parametrize("K", [64, 128, 256])
@pytest.mark.parametrize("tile", [11, 12, 13])
def test_stream_gemm_matches_tiled(K, tile):
    """Streaming kernel (B panel resident in LDS, A straight to registers): forward with the BN
    prologue + column statistics, and data-gradient with the residual addend, against the tiled
    kernel (bit-identical outputs: same k order and rounding) and fp32 statistics."""
    if K == 256 and tile == 13:
        pytest.skip("K=256 streams with panels <= 128")
    lib = G.load()
    torch.manual_seed(5)
    M, N = 3000, 320
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    sc = torch.rand(K, device="cuda") + 0.5
    sh = torch.randn(K, device="cuda")
    ref, _ = lib.gemm_ex(x, K, True, w, K, True, M, N, K, None, False, 1, True, 1, sc, sh, True,
                         False)
    C, st = lib.gemm_ex(x, K, True, w, K, True, M, N, K, None, False, 1, True, tile, sc, sh, True,
                        True)
    torch.testing.assert_close(C, ref, rtol=0, atol=0)
    c = C.float()
    torch.testing.assert_close(st[:, 0].sum(0), c.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(st[:, 1].sum(0), (c * c).sum(0), rtol=1e-4, atol=1e-1)
    # data gradient: dy [M, K] · W [K, N] (N-contiguous B) + addend
    wt = torch.randn(K, N, device="cuda").bfloat16()
    add = torch.randn(M, N, device="cuda").bfloat16()
    ref2 = (lib.gemm_ex(x, K, True, wt, N, False, M, N, K, None, False, 1, True, 1, None, None,
                        True, False)[0].float() + add.float()).bfloat16()
    D, _ = lib.gemm_ex(x, K, True, wt, N, False, M, N, K, None, False, 1, True, tile, None, None,
                       True, False, None, add, False, 0)
    torch.testing.assert_close(D, ref2, rtol=0, atol=0)


@pytest.mark.parametrize("tile", [1, 2, 6, 11, 12])
def test_gemm_masked_addend(tile):
    """dx = dy·W + dres·[bit]: the ReLU-masked shortcut gradient enters through the epilogue."""
    lib = G.load()
    torch.manual_seed(6)
    M, N, K = 2048, 256, 64
    a = torch.randn(M, K, device="cuda").bfloat16()
    wt = torch.randn(K, N, device="cuda").bfloat16()
    add = torch.randn(M, N, device="cuda").bfloat16()
    keep = torch.rand(M, N, device="cuda") > 0.4
    bits = (keep.view(-1, 8).to(torch.uint8) << torch.arange(8, device="cuda",
                                                             dtype=torch.uint8)).sum(1)
    bits = bits.to(torch.uint8)
    base = lib.gemm_ex(a, K, True, wt, N, False, M, N, K, None, False, 1, True, 1, None, None,
                       True, False)[0]
    ref = (base.float() + (add.float() * keep)).bfloat16()
    D = lib.gemm_ex(a, K, True, wt, N, False, M, N, K, None, False, 1, True, tile, None, None,
                    True, False, None, add, False, 0, bits)[0]
    torch.testing.assert_close(D, ref, rtol=0, atol=0)


def _unpack_bits(bits, n):
    b = bits.to(torch.int32)
    out = torch.stack([(b >> k) & 1 for k in range(8)], 1).reshape(-1)[:n]
    return out.bool()


@pytest.mark.parametrize("M,N,K", [(512, 512, 512), (520, 264, 328), (1000, 136, 72),
                                   (256, 1024, 2048), (64, 40, 8)])
@pytest.mark.parametrize("splits", [1, 3])
@pytest.mark.parametrize("tile", ["256x256x64", "256x128x64"])
@pytest.mark.parametrize("kc", [True, False], ids=["kc", "mn"])
def test_gemm_big_tile(M, N, K, splits, tile, kc):
    """256x256 / 256x128 8-wave LDS-DMA kernel (csrc/gemm_big.hip, tiles 21/22), both operands
    K-contiguous (x·Wᵀ) or both MN-contiguous (a weight gradient dYᵀ·X, transposing LDS reads):
    fp32 and bf16 outputs, bias + ReLU, ragged M/N/K edges, split-K, fp32 accumulate."""
    lib = _lib()
    torch.manual_seed(7)
    Am = torch.randn(M, K, device="cuda").bfloat16()
    Bm = torch.randn(N, K, device="cuda").bfloat16()
    A = Am if kc else Am.t().contiguous()              # [M][K] or [K][M]
    B = Bm if kc else Bm.t().contiguous()              # [N][K] or [K][N]
    lda, ldb = (K, K) if kc else (M, N)
    ref = Am.float() @ Bm.float().t()
    C, _ = G.gemm_ex(A, lda, kc, B, ldb, kc, M, N, K, splits=splits, out_bf16=False, tile=tile)
    torch.testing.assert_close(C, ref, rtol=1e-3, atol=1e-2)
    bias = torch.randn(N, device="cuda")
    Y, _ = G.gemm_ex(A, lda, kc, B, ldb, kc, M, N, K, bias=bias, relu=True, splits=splits,
                     tile=tile)
    torch.testing.assert_close(Y.float(), torch.relu(ref + bias), rtol=2e-2, atol=5e-2)
    base = torch.randn(M, N, device="cuda")
    out = base.clone()
    lib.gemm_ex(A, lda, kc, B, ldb, kc, M, N, K, None, False, splits, False, G.TILES[tile], None,
                None, True, False, out, None, True, 0, None)
    torch.testing.assert_close(out, base + ref, rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("tile", ["256x256x64", "256x128x64"])
@pytest.mark.parametrize("kc", [True, False], ids=["kc", "mn"])
def test_gemm_big_tile_bitwise_vs_128(tile, kc):
    """Same per-element k order as the 128x128x64 tile (k ascending in 32-wide MFMA steps):
    the outputs agree exactly."""
    torch.manual_seed(8)
    M, N, K = 768, 512, 640
    Am = torch.randn(M, K, device="cuda").bfloat16()
    Bm = torch.randn(N, K, device="cuda").bfloat16()
    A = Am if kc else Am.t().contiguous()
    B = Bm if kc else Bm.t().contiguous()
    lda, ldb = (K, K) if kc else (M, N)
    c1, _ = G.gemm_ex(A, lda, kc, B, ldb, kc, M, N, K, out_bf16=False, tile=tile)
    c2, _ = G.gemm_ex(A, lda, kc, B, ldb, kc, M, N, K, out_bf16=False, tile="128x128x64")
    torch.testing.assert_close(c1, c2, rtol=0, atol=0)


@pytest.mark.parametrize("M,N,K", [(50176 // 4, 1024, 256), (3000, 264, 136), (70000, 64, 128),
                                   (1000, 2048, 512), (256 * 300, 256, 72)])
@pytest.mark.parametrize("tile", [23, 24])
def test_gemm_persistent_big_tile(M, N, K, tile):
    """Persistent big tiles (csrc/gemm_big.hip k_gemm_bigp, tiles 23/24: one workgroup per CU
    walking several tiles, the next tile's K-tiles 0/1 loaded during the epilogue): bf16 output
    bit-identical to the 128x128x64 tile (plain, + column statistics, + ReLU-masked addend), the
    statistics rows (one per 128 rows) fold to the column sums; ragged M / N / K, T = 2 K-tiles,
    more tiles than CUs."""
    lib = _lib()
    torch.manual_seed(tile + K)
    A = torch.randn(M, K, device="cuda").bfloat16()
    B = torch.randn(N, K, device="cuda").bfloat16()
    add = torch.randn(M, N, device="cuda").bfloat16()
    bits = torch.randint(0, 256, (M * N // 8,), dtype=torch.uint8, device="cuda")
    for stats in (False, True):
        ref, _ = lib.gemm_ex(A, K, True, B, K, True, M, N, K, None, False, 1, True, 2, None, None,
                             True, stats, None, None, False, 0)
        got, st = lib.gemm_ex(A, K, True, B, K, True, M, N, K, None, False, 1, True, tile, None,
                              None, True, stats, None, None, False, 0)
        assert torch.equal(got, ref)
        if stats:
            assert st.shape[0] == -(-M // 128)
            yf = got.float()
            s = st.sum(0)
            torch.testing.assert_close(s[0], yf.sum(0), rtol=1e-3, atol=1e-1)
            torch.testing.assert_close(s[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-1)
    ref = lib.gemm_ex(A, K, True, B, K, True, M, N, K, None, False, 1, True, 2, None, None, True,
                      False, None, add, False, 0, bits)[0]
    got = lib.gemm_ex(A, K, True, B, K, True, M, N, K, None, False, 1, True, tile, None, None,
                      True, False, None, add, False, 0, bits)[0]
    assert torch.equal(got, ref)
    dst = add.clone()                                 # in place: out aliases the addend
    lib.gemm_ex(A, K, True, B, K, True, M, N, K, None, False, 1, True, tile, None, None, True,
                False, dst, dst, False, 0, None)
    ref2 = lib.gemm_ex(A, K, True, B, K, True, M, N, K, None, False, 1, True, 2, None, None, True,
                       False, None, add, False, 0, None)[0]
    assert torch.equal(dst, ref2)


@pytest.mark.parametrize("M,N,K", [(512, 25088 // 8, 4096 // 4), (520, 264, 328), (1000, 136, 72)])
@pytest.mark.parametrize("tile", ["256x256x64", "256x128x64"])
def test_gemm_big_tile_mixed_layout(M, N, K, tile):
    """Big tiles with a K-contiguous A and an N-contiguous B (a data gradient dY·W with W as
    stored): fp32 vs torch with 1 / 3 split-K slices and bit-identical to the 128x128x64 tile."""
    torch.manual_seed(9)
    A = torch.randn(M, K, device="cuda").bfloat16()
    Bkn = torch.randn(K, N, device="cuda").bfloat16()           # [K][N], N-contiguous
    ref = A.float() @ Bkn.float()
    for sp in (1, 3):
        C, _ = G.gemm_ex(A, K, True, Bkn, N, False, M, N, K, splits=sp, out_bf16=False, tile=tile)
        torch.testing.assert_close(C, ref, rtol=1e-3, atol=1e-2)
    c1, _ = G.gemm_ex(A, K, True, Bkn, N, False, M, N, K, out_bf16=False, tile=tile)
    c2, _ = G.gemm_ex(A, K, True, Bkn, N, False, M, N, K, out_bf16=False, tile="128x128x64")
    torch.testing.assert_close(c1, c2, rtol=0, atol=0)


@pytest.mark.parametrize("n,R", [(1000, 49), (4096 * 512, 49), (77, 1), (300, 64)])
def test_sum_repeats_matches_torch(n, R):
    """nn.hip k_sum_repeats (the folded fc1 weight): Σ over the last dim of a 16-bit tensor."""
    torch.manual_seed(5)
    w = torch.randn(n, R, device="cuda").bfloat16()
    got = _lib().sum_repeats(w, R)
    ref = w.float().sum(-1)
    assert got.dtype == torch.bfloat16 and got.shape == (n,)
    torch.testing.assert_close(got.float(), ref, rtol=1e-2, atol=1e-2)


def test_replicated_linear_matches_fp32():
    """ops/gemm.py replicated_linear (the folded fc1 of CIFAR VGG-16) against an fp32 Linear on
    the explicitly repeated input: output, input / weight / bias gradients."""
    torch.manual_seed(4)
    B, C, R, O = 32, 512, 49, 1024
    lin = G.MFMALinear(C * R, O).cuda()
    lin.weight.data = lin.weight.data.bfloat16().float()
    x = torch.randn(B, C, device="cuda").bfloat16().float().requires_grad_()
    xr = x.detach().clone().requires_grad_()
    ref = torch.nn.Linear(C * R, O).cuda()
    ref.load_state_dict(lin.state_dict())
    y = G.replicated_linear(x, lin, R)
    yr = ref(xr.unsqueeze(-1).expand(B, C, R).reshape(B, C * R))
    _close_rel = lambda a, b, tol: float((a.float() - b).norm() / b.norm()) < tol   # noqa: E731
    assert _close_rel(y, yr, 1e-2)
    g = torch.randn_like(yr)
    y.backward(g.to(y.dtype))
    yr.backward(g)
    assert _close_rel(x.grad, xr.grad, 1e-2)
    assert _close_rel(lin.weight.grad, ref.weight.grad, 1e-2)
    assert _close_rel(lin.bias.grad, ref.bias.grad, 1e-2)
    # the weight gradient is the same for every repeat of a feature
    gw = lin.weight.grad.view(O, C, R)
    assert torch.equal(gw, gw[:, :, :1].expand_as(gw))


def test_vgg_replicated_fc1_matches_pool_and_full_gemm(monkeypatch):
    """CIFAR VGG-16 end to end: with the folded fc1 (1x1 feature map, AdaptiveAvgPool2d((7, 7))
    replicating it) the loss matches the pool + full-width GEMM path. (Gradients differ by the
    ReLU-mask flips of near-zero bf16 activations, so they are pinned layer-level above.)"""
    import copy
    from layer_wise_aaai20_amd.models import cifar as CM
    from layer_wise_aaai20_amd.ops.conv import fuse_convs
    torch.manual_seed(3)
    base = CM.vgg16()
    fuse_convs(base)
    G.fuse_linears(base)
    base = base.cuda().to(memory_format=torch.channels_last).eval()       # eval: no dropout
    x = torch.randn(8, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    t = torch.randint(0, 10, (8,), device="cuda")
    loss = {}
    for fold in (True, False):
        monkeypatch.setattr(CM, "_VGG_FOLD", fold)
        m = copy.deepcopy(base)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = m({"input": x, "target": t})
        loss[fold] = float(out["loss"].float().sum())
        out["loss"].float().sum().backward()
        assert m.classifier[0].weight.grad is not None
    assert abs(loss[True] - loss[False]) < 1e-2 * abs(loss[False]), loss


def test_linear_with_unaligned_in_features_runs_padded_on_mfma():
    """in_features % 8 != 0: both operands zero-padded to a multiple of 8 and run on the MFMA
    GEMM (no vendor fallback); forward and gradients vs fp32 torch, gradient shapes unpadded."""
    torch.manual_seed(9)
    x = torch.randn(96, 100, device="cuda").bfloat16().float().requires_grad_()
    w = torch.randn(40, 100, device="cuda").bfloat16().float().requires_grad_()
    b = torch.randn(40, device="cuda").requires_grad_()
    y = G.mfma_linear(x.bfloat16(), w.bfloat16(), b)
    xr, wr, br = (t.detach().clone().requires_grad_() for t in (x, w, b))
    yr = xr @ wr.t() + br
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=5e-2)
    g = torch.randn_like(yr).bfloat16()
    y.backward(g)
    yr.backward(g.float())
    assert x.grad.shape == (96, 100) and w.grad.shape == (40, 100)
    torch.testing.assert_close(x.grad, xr.grad, rtol=3e-2, atol=1e-1)
    torch.testing.assert_close(w.grad, wr.grad, rtol=3e-2, atol=1e-1)
