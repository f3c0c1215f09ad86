"""Numerics of the CDNA4 HIP kernels against plain PyTorch fp32 references of the same op."""
import pytest
import torch

from netsdb_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _ref_gemm(A, B, bias=None, mode=0, act=0):
    v = A.float() @ B.float().transpose(-1, -2)
    if bias is not None:
        v = v + (bias.unsqueeze(-1) if mode == 1 else bias.unsqueeze(-2))
    return ops._apply_act(v, act)


def _close(x, ref, tol=2e-2):
    err = (x.float() - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    assert err <= tol * scale, f"max err {err} vs scale {scale}"


def test_gemm_identity_asymmetric():
    # A = I with an asymmetric B catches a transposed C-write (cdna guide §3)
    n = 256
    A = torch.eye(n, device=DEV, dtype=torch.bfloat16)
    B = (torch.arange(n * n, device=DEV, dtype=torch.float32).reshape(n, n) % 97 - 48).to(torch.bfloat16)
    C = ops.gemm_nt(A, B, out_dtype=torch.float32)
    torch.testing.assert_close(C, B.float().t().contiguous(), rtol=0, atol=0)


@pytest.fixture(params=[None, 0, 2, 3, 4], ids=["auto", "tile128", "tile256_8ph", "stream256x128", "stream128x256"])
def gemm_cfg(request):
    """Per-call tile config (ops.gemm_nt(cfg=...)): the production configs of the kernel library."""
    return request.param


@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (1000, 1000, 4096), (77, 300, 520), (513, 129, 8), (2048, 64, 1024),
                                   (600, 520, 2056), (256, 256, 64), (1024, 768, 8192), (300, 1000, 576)])
@pytest.mark.parametrize("splits", [0, 1, 3])
def test_gemm_shapes(M, N, K, splits, gemm_cfg):
    torch.manual_seed(0)
    A = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    B = torch.randn(N, K, device=DEV).to(torch.bfloat16)
    C = ops.gemm_nt(A, B, out_dtype=torch.float32, splits=splits, cfg=gemm_cfg)
    _close(C, _ref_gemm(A, B), tol=1e-2)


@pytest.mark.parametrize("mode,act", [(1, ops.ACT_RELU), (2, ops.ACT_SIGMOID), (2, ops.ACT_NONE), (1, ops.ACT_EXP)])
@pytest.mark.parametrize("splits", [1, 4])
def test_gemm_epilogue(mode, act, splits, gemm_cfg):
    torch.manual_seed(1)
    M, N, K = 300, 200, 640
    A = (torch.randn(M, K, device=DEV) * 0.05).to(torch.bfloat16)
    B = (torch.randn(N, K, device=DEV) * 0.05).to(torch.bfloat16)
    bias = torch.randn(M if mode == 1 else N, device=DEV)
    C = ops.gemm_nt(A, B, bias=bias, bias_mode=mode, act=act, out_dtype=torch.float32, splits=splits, cfg=gemm_cfg)
    _close(C, _ref_gemm(A, B, bias, mode, act), tol=1e-2)
    Cb = ops.gemm_nt(A, B, bias=bias, bias_mode=mode, act=act, out_dtype=torch.bfloat16, splits=splits, cfg=gemm_cfg)
    _close(Cb, _ref_gemm(A, B, bias, mode, act), tol=2e-2)


@pytest.mark.parametrize("M,N,K", [(300, 200, 640), (1000, 1030, 1000), (257, 514, 64)])
@pytest.mark.parametrize("mode,act,dropout", [(0, ops.ACT_NONE, 0.0), (1, ops.ACT_RELU, 0.0), (2, ops.ACT_EXP, 0.0),
                                              (2, ops.ACT_SIGMOID, 0.3)])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_gemm_8ph_direct_epilogue_matches_lds_staged(M, N, K, mode, act, dropout, out_dtype):
    """The 8-phase kernel's direct register epilogue (epi=1, default for unsplit launches) and its LDS-staged
    epilogue (epi=0) write the same values (same fp32 math, same dropout hash), ragged edges included; both
    against the fp32 reference."""
    torch.manual_seed(7)
    A = (torch.randn(M, K, device=DEV) * 0.05).to(torch.bfloat16)
    B = (torch.randn(N, K, device=DEV) * 0.05).to(torch.bfloat16)
    bias = torch.randn(M if mode == 1 else N, device=DEV) if mode else None
    kw = dict(bias=bias, bias_mode=mode, act=act, out_dtype=out_dtype, dropout=dropout, seed=99, splits=1, cfg=2)
    Cd = ops.gemm_nt(A, B, epi=1, **kw)
    Cl = ops.gemm_nt(A, B, epi=0, **kw)
    torch.testing.assert_close(Cd, Cl, rtol=0, atol=0)
    if dropout == 0.0:
        _close(Cd, _ref_gemm(A, B, bias, mode, act), tol=2e-2)
    # ldc-padded output (a column slice of a wider buffer), as the FF output layer writes it
    wide = torch.full((M, (N + 63) // 64 * 64), -7.0, device=DEV, dtype=out_dtype)
    view = wide[:, :N]
    ops.gemm_nt(A, B, out=view, epi=1, **kw)
    torch.testing.assert_close(view, Cl, rtol=0, atol=0)
    assert (wide[:, N:] == -7.0).all()


def test_gemm_8ph_mfma32_identity_asymmetric():
    """The 32x32x16 main loop (mfma=32): A = I with an asymmetric B catches a transposed C-write or a wrong k
    permutation between the two operands' fragments."""
    n = 512
    A = torch.eye(n, device=DEV, dtype=torch.bfloat16)
    B = (torch.arange(n * n, device=DEV, dtype=torch.float32).reshape(n, n) % 97 - 48).to(torch.bfloat16)
    C = ops.gemm_nt(A, B, out_dtype=torch.float32, cfg=2, splits=1, mfma=32)
    torch.testing.assert_close(C, B.float().t().contiguous(), rtol=0, atol=0)
    Ct = ops.gemm_nt(B, A, out_dtype=torch.float32, cfg=2, splits=1, mfma=32)
    torch.testing.assert_close(Ct, B.float(), rtol=0, atol=0)


@pytest.mark.parametrize("M,N,K", [(1000, 1000, 6400), (300, 200, 640), (1000, 1030, 1000), (257, 514, 72),
                                   (256, 256, 64), (513, 260, 8200)])
@pytest.mark.parametrize("splits", [1, 3, 16])
def test_gemm_8ph_mfma32_exact_vs_mfma16(M, N, K, splits):
    """Small-integer operands make every partial sum exact in f32, so the 32x32x16 and 16x16x32 main loops must
    agree bit for bit (split-K slabs + reducer, ragged M / N / K edges), and both equal the f32 reference."""
    torch.manual_seed(21)
    A = torch.randint(-3, 4, (M, K), device=DEV).to(torch.bfloat16)
    B = torch.randint(-3, 4, (N, K), device=DEV).to(torch.bfloat16)
    c32 = ops.gemm_nt(A, B, out_dtype=torch.float32, cfg=2, splits=splits, mfma=32)
    c16 = ops.gemm_nt(A, B, out_dtype=torch.float32, cfg=2, splits=splits, mfma=16)
    torch.testing.assert_close(c32, c16, rtol=0, atol=0)
    torch.testing.assert_close(c32, _ref_gemm(A, B), rtol=0, atol=0)


@pytest.mark.parametrize("mode,act,dropout", [(0, ops.ACT_NONE, 0.0), (1, ops.ACT_RELU, 0.0), (2, ops.ACT_EXP, 0.0),
                                              (2, ops.ACT_SIGMOID, 0.3), (1, ops.ACT_RELU, 0.5)])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("splits", [1, 4])
def test_gemm_8ph_mfma32_epilogue(mode, act, dropout, out_dtype, splits):
    """The 32x32x16 loop's register epilogue (bias per row / column, activations, dropout hash, bf16 packing) and
    its split-K slabs against the fp32 reference, with the dropout mask equal to the 16x16x32 loop's."""
    torch.manual_seed(8)
    M, N, K = 1000, 1030, 1024
    A = (torch.randn(M, K, device=DEV) * 0.05).to(torch.bfloat16)
    B = (torch.randn(N, K, device=DEV) * 0.05).to(torch.bfloat16)
    bias = torch.randn(M if mode == 1 else N, device=DEV) if mode else None
    kw = dict(bias=bias, bias_mode=mode, act=act, out_dtype=out_dtype, dropout=dropout, seed=5, splits=splits, cfg=2)
    c32 = ops.gemm_nt(A, B, mfma=32, **kw)
    c16 = ops.gemm_nt(A, B, mfma=16, **kw)
    assert torch.equal(c32 == 0, c16 == 0) or act == ops.ACT_RELU
    if dropout == 0.0:
        _close(c32, _ref_gemm(A, B, bias, mode, act), tol=2e-2)
    _close(c32, c16.float(), tol=2e-2)


def test_gemm_8ph_mfma32_ff_layer1_shape():
    """The headline layer-1 shape class (M = N = 1000, K long, split-K 16) on the 32x32x16 loop vs fp32."""
    torch.manual_seed(9)
    M, N, K = 1000, 1000, 65536
    A = (torch.rand(M, K, device=DEV) - 0.5).to(torch.bfloat16)
    B = (torch.rand(N, K, device=DEV) - 0.5).to(torch.bfloat16)
    C = ops.gemm_nt(A, B, out_dtype=torch.float32, cfg=2, mfma=32)
    _close(C, _ref_gemm(A, B), tol=1e-2)


@pytest.mark.parametrize("M,N,K,splits", [(1000, 1000, 65536, 16), (513, 260, 8200, 3), (1100, 1028, 64000, 32),
                                          (1000, 1000, 640, 5), (300, 1028, 64000, 32)])
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
def test_gemm_8ph_split_k_fixup_bit_exact(M, N, K, splits, out_dtype):
    """The split-K reduction inside the 8-phase launch (splits of a tile meet, each reduces its rows) is bit-identical
    to the separate reducer — the same slabs summed in split order, the same epilogue (bias, relu, dropout) — on
    ragged M / N edges, three launches in a row (the arrival / departure words are re-zeroed by each launch). Narrow
    outputs with many splits (300 x 1028 at 32) keep the wide reducer: equal by construction there."""
    torch.manual_seed(13)
    A = (torch.rand(M, K, device=DEV) - 0.5).to(torch.bfloat16)
    B = (torch.rand(N, K, device=DEV) - 0.5).to(torch.bfloat16)
    bias = torch.rand(N, device=DEV) - 0.5
    kw = dict(bias=bias, bias_mode=ops.BIAS_COL, act=ops.ACT_RELU, dropout=0.5, seed=3, out_dtype=out_dtype, cfg=2,
              splits=splits)
    ref = ops.gemm_nt(A, B, fixup=0, **kw)
    for _ in range(3):
        got = ops.gemm_nt(A, B, fixup=1, **kw)
        assert torch.equal(got, ref)
    _close(ops.gemm_nt(A, B, fixup=1, out_dtype=torch.float32, cfg=2, splits=splits), _ref_gemm(A, B), tol=1e-2)


def test_gemm_batched_strided(gemm_cfg):
    torch.manual_seed(2)
    A = torch.randn(3, 130, 200, device=DEV).to(torch.bfloat16)[:, :, :192]   # row stride 200 > K
    B = torch.randn(3, 70, 192, device=DEV).to(torch.bfloat16)
    C = ops.gemm_nt(A, B, out_dtype=torch.float32, cfg=gemm_cfg)
    _close(C, _ref_gemm(A, B), tol=1e-2)


@pytest.mark.parametrize("M,N,K,batch", [(500, 100, 90000, 1), (100, 500, 40000, 1), (500, 100, 10000, 4),
                                         (1000, 64, 60000, 1), (6000, 100, 20000, 1), (300, 8, 20000, 1),
                                         (40, 2000, 17000, 1)])
def test_gemm_stream_skinny_long_k(M, N, K, batch):
    """The skinny long-K stream tiles (cfg 3: 256x128, cfg 4: 128x256; the dedup scoring shapes, scaled down)
    against the fp32 reference and bit-exact against each other's split partition: same k-tiles, same order."""
    torch.manual_seed(11)
    shp = (batch,) if batch > 1 else ()
    A = (torch.rand(*shp, M, K, device=DEV) - 0.5).to(torch.bfloat16)
    B = (torch.rand(*shp, N, K, device=DEV) - 0.5).to(torch.bfloat16)
    ref = _ref_gemm(A, B)
    for cfg in (3, 4, 5, 6, None):
        C = ops.gemm_nt(A, B, out_dtype=torch.float32, cfg=cfg)
        _close(C, ref, tol=1e-2)


def test_gemm_accumulate(gemm_cfg):
    torch.manual_seed(5)
    A = torch.randn(300, 256, device=DEV).to(torch.bfloat16)
    B = torch.randn(280, 256, device=DEV).to(torch.bfloat16)
    C = torch.randn(300, 280, device=DEV)
    ref = C + _ref_gemm(A, B)
    ops.gemm_nt(A, B, out=C, out_dtype=torch.float32, accumulate=True, cfg=gemm_cfg)
    _close(C, ref, tol=1e-2)


def test_gemm_dropout_matches_host_rng():
    torch.manual_seed(3)
    A = torch.randn(64, 64, device=DEV).to(torch.bfloat16)
    B = torch.randn(32, 64, device=DEV).to(torch.bfloat16)
    C = ops.gemm_nt(A, B, out_dtype=torch.float32, dropout=0.5, seed=1234, splits=1)
    ref = ops.gemm_nt(A.cpu(), B.cpu(), out_dtype=torch.float32, dropout=0.5, seed=1234)
    assert torch.equal(C.cpu() == 0, ref == 0)
    _close(C.cpu(), ref, tol=1e-2)


@pytest.fixture(params=[0, 1], ids=["auto", "generic"])
def conv_generic(request):
    with ops.kernel_options(conv_generic=bool(request.param)):
        yield request.param


@pytest.mark.parametrize("cfg", [
    dict(N=2, C=3, H=20, W=20, OC=8, KH=7, KW=7, stride=1, pad=0),     # the memfuse 7x7x3 shape, small
    dict(N=3, C=3, H=30, W=112, OC=64, KH=7, KW=7, stride=1, pad=0),   # row kernel: headline geometry
    dict(N=2, C=2, H=13, W=16, OC=70, KH=5, KW=3, stride=1, pad=0),    # row kernel: 2 oc tiles, OH % 4 != 0
    dict(N=1, C=1, H=9, W=128, OC=16, KH=8, KW=8, stride=1, pad=0),    # row kernel: KW = 8, OW = 121
    dict(N=1, C=64, H=14, W=14, OC=70, KH=3, KW=3, stride=2, pad=1),   # K=576 > one LDS K chunk, OC edge
    dict(N=3, C=16, H=9, W=11, OC=64, KH=1, KW=1, stride=1, pad=0),
])
@pytest.mark.parametrize("nchw", [False, True])
def test_conv2d(cfg, nchw, conv_generic):
    torch.manual_seed(4)
    X = torch.randn(cfg["N"], cfg["C"], cfg["H"], cfg["W"], device=DEV).to(torch.bfloat16)
    K = cfg["C"] * cfg["KH"] * cfg["KW"]
    Wt = ops.pad_k(torch.randn(cfg["OC"], K, device=DEV) * 0.1).to(torch.bfloat16).contiguous()
    bias = torch.randn(cfg["OC"], device=DEV)
    y = ops.conv2d(X, Wt, bias, cfg["KH"], cfg["KW"], cfg["stride"], cfg["pad"], act=ops.ACT_RELU, nchw_out=nchw,
                   out_dtype=torch.float32)
    ref = ops.conv2d(X.cpu(), Wt.cpu(), bias.cpu(), cfg["KH"], cfg["KW"], cfg["stride"], cfg["pad"],
                     act=ops.ACT_RELU, nchw_out=nchw, out_dtype=torch.float32)
    _close(y.cpu(), ref, tol=1e-2)


def test_im2col():
    X = torch.randn(2, 3, 12, 10, device=DEV).to(torch.bfloat16)
    a = ops.im2col(X, 3, 3, 1, 1)
    b = ops.im2col(X.cpu(), 3, 3, 1, 1)
    torch.testing.assert_close(a.cpu().float(), b.float())


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_softmax_rows(dt):
    X = (torch.randn(37, 14588, device=DEV) * 3).to(dt)
    bias = torch.randn(14588, device=DEV)
    y = ops.softmax_rows(X, bias)
    _close(y, torch.softmax(X.float() + bias, -1), tol=1e-3)
    assert torch.allclose(y.sum(-1), torch.ones(37, device=DEV), atol=1e-4)


@pytest.mark.parametrize("R,N", [(37, 14588), (5, 1000), (3, 130), (4, 50000), (2, 7)])
@pytest.mark.parametrize("out_f32", [True, False])
def test_row_normalize(R, N, out_f32):
    X = torch.rand(R, N, device=DEV) + 0.1
    y = ops.row_normalize(X, out_dtype=torch.float32 if out_f32 else torch.bfloat16)
    _close(y, X / X.sum(-1, keepdim=True), tol=1e-2 if not out_f32 else 1e-5)


@pytest.mark.parametrize("n0,n1", [(0, 256), (3, 301), (128, 1000), (1, 2)])
def test_gemm_out_column_slice(n0, n1):
    # C[:, n0:n1] views (ldc != N, unaligned base): the distributed N-chunk pipeline writes these
    torch.manual_seed(6)
    A = torch.randn(200, 320, device=DEV).to(torch.bfloat16)
    B = torch.randn(1000, 320, device=DEV).to(torch.bfloat16)
    bias = torch.randn(1000, device=DEV)
    for dt in (torch.float32, torch.bfloat16):
        C = torch.zeros(200, 1000, device=DEV, dtype=dt)
        ops.gemm_nt(A, B[n0:n1], bias[n0:n1], ops.BIAS_COL, ops.ACT_RELU, out_dtype=dt, out=C[:, n0:n1])
        ref = torch.zeros(200, 1000, device=DEV)
        ref[:, n0:n1] = _ref_gemm(A, B[n0:n1], bias[n0:n1], 2, ops.ACT_RELU)
        _close(C, ref, tol=2e-2)
        assert C[:, :n0].abs().sum() == 0 and C[:, n1:].abs().sum() == 0


def test_bias_act_and_lstm_and_embedding():
    X = torch.randn(33, 65, device=DEV)
    b = torch.randn(33, device=DEV)
    _close(ops.bias_act(X, b, ops.BIAS_ROW, ops.ACT_RELU, out_dtype=torch.float32), torch.relu(X + b[:, None]), 1e-6)
    g = torch.randn(16, 4 * 40, device=DEV)
    c0 = torch.randn(16, 40, device=DEV)
    h, c = ops.lstm_cell(g, c0)
    hr, cr = ops.lstm_cell(g.cpu(), c0.cpu())
    _close(h.cpu(), hr, 1e-5)
    _close(c.cpu(), cr, 1e-5)
    table = torch.randn(1000, 300, device=DEV)
    idx = torch.randint(0, 1000, (50,), device=DEV)
    offs = torch.tensor([0, 5, 5, 20, 50], device=DEV)
    e = ops.embedding_bag(table, idx, offs, mode="mean")
    er = ops.embedding_bag(table.cpu(), idx.cpu(), offs.cpu(), mode="mean")
    _close(e.cpu(), er, 1e-5)


@pytest.mark.parametrize("S,N,segk,M", [(2, 300, 128, 200), (4, 1000, 320, 256), (8, 777, 64, 130)])
@pytest.mark.parametrize("out_f32", [True, False])
def test_gemm_segmented_b_in_place(S, N, segk, M, out_f32):
    """The all-gathered [S, N, seg_k] chunk consumed in place (K segment s at B + s*N*seg_k) vs the
    permuted K-contiguous panel: the distributed all-gather pipeline's GEMM."""
    torch.manual_seed(9)
    A = torch.randn(M, S * segk, device=DEV).to(torch.bfloat16)
    Bg = torch.randn(S, N, segk, device=DEV).to(torch.bfloat16)
    bias = torch.randn(N, device=DEV)
    dt = torch.float32 if out_f32 else torch.bfloat16
    C = ops.gemm_nt_segmented(A, Bg, bias, ops.BIAS_COL, ops.ACT_RELU, out_dtype=dt)
    ref = _ref_gemm(A, Bg.permute(1, 0, 2).reshape(N, S * segk), bias, 2, ops.ACT_RELU)
    _close(C, ref, tol=1e-2 if out_f32 else 2e-2)


def test_gemm_bias_matrix_epilogue():
    torch.manual_seed(10)
    A = torch.randn(300, 256, device=DEV).to(torch.bfloat16)
    B = torch.randn(500, 256, device=DEV).to(torch.bfloat16)
    bm = torch.randn(300, 500, device=DEV)
    for splits in (1, 3):
        C = ops.gemm_nt(A, B, bm, ops.BIAS_MAT, ops.ACT_SIGMOID, out_dtype=torch.float32, splits=splits)
        _close(C, torch.sigmoid(A.float() @ B.float().t() + bm), tol=1e-2)


def test_lstm_elementwise_kernels():
    f, cp, i, g = (torch.randn(130, 77, device=DEV) for _ in range(4))
    _close(ops.lstm_two_sum(f, cp, i, g), f * cp + i * g, 1e-6)
    _close(ops.lstm_hidden(f, cp), f * torch.tanh(cp), 1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(500, 100, 100000), (500, 100, 900000), (64, 48, 65536)])
def test_gemm_narrow_many_splits_wide_reducer(M, N, K):
    """Small M x N with huge K (dedup scoring): many split-K slices reduced by the wide reducer."""
    g = torch.Generator(device="cuda:0").manual_seed(5)
    A = (torch.randn(M, K, device="cuda:0", generator=g) * 0.05).to(torch.bfloat16)
    B = (torch.randn(N, K, device="cuda:0", generator=g) * 0.05).to(torch.bfloat16)
    assert ops.gemm_splits(M, N, K) >= 8
    bias = torch.randn(M, N, device="cuda:0")
    C = ops.gemm_nt(A, B, bias, ops.BIAS_MAT, out_dtype=torch.float32)
    ref = A.float() @ B.float().t() + bias
    assert (C - ref).abs().max().item() / ref.abs().max().item() < 1e-4


@pytest.mark.gpu
def test_gemm_batched_broadcast_b_and_bias_matrix():
    """Batched private-column scoring: B broadcast over the batch (stride 0), 2-D bias matrix broadcast."""
    g = torch.Generator(device="cuda:0").manual_seed(6)
    A = (torch.randn(5, 300, 20000, device="cuda:0", generator=g) * 0.05).to(torch.bfloat16)
    X = (torch.randn(100, 20000, device="cuda:0", generator=g) * 0.05).to(torch.bfloat16)
    P = torch.randn(300, 100, device="cuda:0")
    Y = ops.gemm_nt(A, X.unsqueeze(0).expand(5, -1, -1), P, ops.BIAS_MAT, out_dtype=torch.float32)
    ref = A.float() @ X.float().t() + P
    assert (Y - ref).abs().max().item() / ref.abs().max().item() < 1e-4


@pytest.mark.parametrize("rowfull,blocks", [(0, 512), (1, 512), (5, 512), (5, 3)],
                         ids=["rows", "rowfull", "warpspec", "warpspec-persistent"])
@pytest.mark.parametrize("cfg", [
    dict(N=3, C=3, H=30, W=112, OC=64, KH=7, KW=7),    # headline geometry (7 pixel tiles per row)
    dict(N=2, C=2, H=14, W=104, OC=70, KH=5, KW=3),    # OW = 102, partial second oc tile, OH % 4 == 2
    dict(N=1, C=3, H=21, W=104, OC=16, KH=7, KW=7),    # OW = 98, one partial oc tile
])
def test_conv2d_rows_bf16_nchw(cfg, rowfull, blocks):
    """The LDS-staged bf16 NCHW output path (what the conv2d job runs): the two-pass row kernel, the full-row
    kernel (1 wave/SIMD, stores pipelined under the MFMAs) and the warp-specialised kernel (compute + store waves;
    with 3 persistent blocks every block walks several row groups) vs the fp32 reference, with a relu epilogue."""
    torch.manual_seed(5)
    X = torch.randn(cfg["N"], cfg["C"], cfg["H"], cfg["W"], device=DEV).to(torch.bfloat16)
    K = cfg["C"] * cfg["KH"] * cfg["KW"]
    Wt = ops.pad_k(torch.randn(cfg["OC"], K, device=DEV) * 0.1).to(torch.bfloat16).contiguous()
    bias = torch.randn(cfg["OC"], device=DEV)
    with ops.kernel_options(conv_kernel=rowfull, conv_blocks=blocks):
        y = ops.conv2d(X, Wt, bias, cfg["KH"], cfg["KW"], 1, 0, act=ops.ACT_RELU, nchw_out=True)
        torch.cuda.synchronize()
    assert y.dtype == torch.bfloat16
    ref = ops.conv2d(X.cpu(), Wt.cpu(), bias.cpu(), cfg["KH"], cfg["KW"], 1, 0, act=ops.ACT_RELU, nchw_out=True,
                     out_dtype=torch.float32)
    _close(y.float().cpu(), ref, tol=1e-2)
