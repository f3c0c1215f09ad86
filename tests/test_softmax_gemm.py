"""Fused, max-subtracted softmax in the GEMM epilogue (FFOutputLayer over FFTransposeBiasSum scores:
src/FF/headers/FFOutputLayer.h, FFRowAggregate.h) vs a plain fp32 PyTorch softmax.

The GPU kernel exchanges per-row (max, sum exp) partials across the workgroups of a row-block; the tests
cover both axes (rows of C, and columns of C when the planner computed C^T), ragged tiles, the headline
FF output-layer shape (1000 x 14588 x 1000), logits far past exp's f32 range (the reference's
exp(x + b) / rowsum overflows there), the timed-out fallback path through the fix-up kernel, and the
engine lowering (fused_ops records softmax_epilogue[gemm])."""
import tempfile

import pytest
import torch

from netsdb_amd import _ext, ops


def _ref(A, B, bias, mode, axis, alpha=1.0):
    v = (A.float() @ B.float().t()) * alpha
    if bias is not None:
        v = v + (bias.float().unsqueeze(1) if mode == ops.BIAS_ROW else bias.float().unsqueeze(0))
    return torch.softmax(v, dim=1 if axis == 1 else 0)


def test_single_job_ff_matches_two_job_cpu(tmp_path):
    """inference_unit(single_job=True) == the reference's two-job form; the fuser sees the softmax as the
    GEMM's only consumer (the precondition of the GPU epilogue fusion)."""
    from netsdb_amd.client import PDBClient
    from netsdb_amd.models import ff
    from netsdb_amd.models.blocks import to_tensor
    from netsdb_amd.query_planning import fusion

    seen = []
    orig = fusion.SoftmaxNode.eval

    def spy(self, engine):
        seen.append((type(self.x).__name__, self.x.uses, getattr(self.x, "act", None)))
        return orig(self, engine)

    fusion.SoftmaxNode.eval = spy
    try:
        c = PDBClient(root=str(tmp_path), device="cpu")
        ff.load_model(c, "ff", 40, 96, 48, 24, 16, 32, dtype=torch.float32)
        ff.inference_unit(c, "ff", "w1", "wo", "inputs", "b1", "bo", "out1")
        a = to_tensor(c, "ff", "out1")
        ff.inference_unit(c, "ff", "w1", "wo", "inputs", "b1", "bo", "out2", single_job=True)
        b = to_tensor(c, "ff", "out2")
    finally:
        fusion.SoftmaxNode.eval = orig
    torch.testing.assert_close(a, b)
    assert ("MatmulNode", 1, "exp") in seen, seen


def test_softmax_gemm_cpu_oracle_is_safe():
    """The CPU path of the op is the max-subtracted softmax (finite for logits past 88)."""
    g = torch.Generator().manual_seed(0)
    A = torch.randn(7, 16, generator=g) * 30
    B = torch.randn(9, 16, generator=g) * 30
    bias = torch.randn(9, generator=g)
    y = ops.gemm_nt_softmax(A, B, bias, ops.BIAS_COL, axis=1)
    assert torch.isfinite(y).all()
    torch.testing.assert_close(y.sum(1), torch.ones(7))
    torch.testing.assert_close(y, _ref(A, B, bias, ops.BIAS_COL, 1))
    y2 = ops.gemm_nt_softmax(A, B, None, axis=2)
    torch.testing.assert_close(y2.sum(0), torch.ones(9))


@pytest.mark.gpu
@pytest.mark.parametrize("epi", [None, 0], ids=["direct", "lds"])
@pytest.mark.parametrize("axis", [1, 2])
@pytest.mark.parametrize("shape,mode", [((300, 700, 96), ops.BIAS_COL), ((777, 555, 4104), ops.BIAS_ROW),
                                        ((256, 256, 64), None), ((1000, 14588, 1000), ops.BIAS_COL),
                                        ((300, 701, 64), ops.BIAS_COL), ((300, 16700, 64), ops.BIAS_COL),
                                        ((16700, 300, 64), ops.BIAS_ROW)])
def test_softmax_gemm_vs_fp32(shape, mode, axis, epi):
    """Direct register stores (C rows 16-B aligned; N = 701 falls back to the LDS-staged store) and the
    LDS-staged final store."""
    M, N, K = shape
    g = torch.Generator(device="cuda:0").manual_seed(1)
    A = (torch.rand(M, K, device="cuda:0", generator=g) * 0.2).to(torch.bfloat16)
    B = (torch.randn(N, K, device="cuda:0", generator=g) / K ** 0.5).to(torch.bfloat16)
    bias = None if mode is None else torch.randn(M if mode == ops.BIAS_ROW else N, device="cuda:0", generator=g)
    y = ops.gemm_nt_softmax(A, B, bias, mode or ops.BIAS_NONE, axis=axis, epi=epi)
    ref = _ref(A, B, bias, mode, axis)
    assert y.shape == (M, N) and y.dtype == torch.float32
    err = ((y - ref).abs().max() / ref.abs().max()).item()
    assert err < 2e-5, err
    s = y.sum(1 if axis == 1 else 0)
    torch.testing.assert_close(s, torch.ones_like(s), atol=1e-4, rtol=0)


@pytest.mark.gpu
def test_softmax_gemm_large_logits_stay_finite():
    """Logits of +-300: exp overflows f32 (the unfused exp -> row-normalise path returns inf/NaN)."""
    M, N, K = 512, 1300, 256
    g = torch.Generator(device="cuda:0").manual_seed(2)
    A = torch.randn(M, K, device="cuda:0", generator=g).to(torch.bfloat16)
    B = (torch.randn(N, K, device="cuda:0", generator=g) * 20.0).to(torch.bfloat16)
    y = ops.gemm_nt_softmax(A, B, None, axis=1)
    ref = _ref(A, B, None, None, 1)
    assert torch.isfinite(y).all()
    assert (y - ref).abs().max().item() < 1e-2          # peaked rows: bf16-operand logit error x ~300
    naive = ops.gemm_nt(A, B, act=ops.ACT_EXP, out_dtype=torch.float32)
    assert not torch.isfinite(naive).all()       # what the max-subtraction protects against


@pytest.mark.gpu
@pytest.mark.parametrize("axis", [1, 2])
def test_softmax_gemm_fallback_fixup(axis):
    """Every tile takes the timed-out path (diag 4): it writes exp(x - m_tile), and the last tile of its group to
    depart rescales it by exp(m_tile - M) / S inside the same launch (no fix-up kernel); the result must still
    match, and the following launches (normal and timed-out, alternating) must see zeroed counters / flags."""
    M, N, K = 600, 1100, 320
    g = torch.Generator(device="cuda:0").manual_seed(3)
    A = torch.randn(M, K, device="cuda:0", generator=g).to(torch.bfloat16)
    B = (torch.randn(N, K, device="cuda:0", generator=g) * 0.1).to(torch.bfloat16)
    bias = torch.randn(N, device="cuda:0", generator=g)
    y = ops.gemm_nt_softmax(A, B, bias, ops.BIAS_COL, axis=axis, force_fallback=True)
    ref = _ref(A, B, bias, ops.BIAS_COL, axis)
    assert (y - ref).abs().max().item() / ref.abs().max().item() < 2e-5
    for fb in (False, True, False):
        y2 = ops.gemm_nt_softmax(A, B, bias, ops.BIAS_COL, axis=axis, force_fallback=fb)
        torch.testing.assert_close(y2, y, atol=1e-6, rtol=1e-5)


@pytest.mark.gpu
def test_ff_engine_fuses_softmax_into_gemm_epilogue():
    """The single-job FF graph (FFTransposeMult + FFAggMatrix + FFTransposeBiasSum(exp) + FFRowAggregate +
    FFOutputLayer) lowers its output layer to one GEMM with the normalisation in its epilogue."""
    from netsdb_amd.client import PDBClient
    from netsdb_amd.models import ff
    from netsdb_amd.models.blocks import to_tensor

    c = PDBClient(root=tempfile.mkdtemp(), device="cuda:0")
    ff.load_model(c, "ff", 200, 512, 256, 700, 64, 128, seed=0)
    res = ff.inference_unit(c, "ff", "w1", "wo", "inputs", "b1", "bo", "output", single_job=True)
    fused = [op for j in res["jobs"] for op in j.get("fused_ops", [])]
    assert "softmax_epilogue[gemm]" in fused, fused
    out = to_tensor(c, "ff", "output").float()
    gt = lambda n: to_tensor(c, "ff", n)  # noqa: E731
    ref = ff.reference_inference(gt("inputs"), gt("w1"), gt("b1"), gt("wo"), gt("bo"))
    assert (out - ref).abs().max().item() < 2e-3
    torch.testing.assert_close(out.sum(1), torch.ones(out.shape[0], device=out.device), atol=1e-4, rtol=0)


@pytest.mark.gpu
def test_softmax_gemm_beside_long_gemm_gpu():
    """The fused softmax needs every tile of a row-block resident at once. Here it is launched on a second stream
    right behind a long split-K GEMM that holds most CUs, so some of its 228 tiles (FF output shape) get CUs only as
    the GEMM's workgroups finish: tiles whose bounded poll runs out write exp(x - m_tile) and depart flagged, and
    the last tile to depart rescales them. Whatever the interleaving, the result is exact and the launch ends."""
    from netsdb_amd import _ext
    from netsdb_amd.execution.streams import JobStreams

    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(11)
    M, N, K = 1000, 14588, 1000
    A = torch.empty(M, K, device=dev).uniform_(0, 1, generator=g).to(torch.bfloat16)
    B = (torch.empty(N, K, device=dev).uniform_(-1, 1, generator=g) * 0.055).to(torch.bfloat16)
    bias = torch.empty(N, device=dev).uniform_(-0.1, 0.1, generator=g)
    GA = torch.empty(1024, 1 << 20, device=dev).uniform_(-1, 1, generator=g).to(torch.bfloat16)
    GB = (torch.empty(1024, 1 << 20, device=dev).uniform_(-1, 1, generator=g) * 1e-3).to(torch.bfloat16)
    ref = _ref(A, B, bias, ops.BIAS_COL, 1)
    torch.cuda.synchronize()
    tiles = ((M + 255) // 256) * ((N + 255) // 256)
    st = torch.zeros(tiles * 8, dtype=torch.int64, device=dev)
    js = JobStreams(dev, lanes=1)
    for rep in range(3):
        C = ops.gemm_nt(GA, GB, out_dtype=torch.float32)          # ~4 ms, 192 workgroups
        h = js.submit(lambda: _ext.hip().gemm_nt_softmax(A, B, bias, ops.BIAS_COL, 1, None, 1.0, False, -1, st),
                      independent=True)
        y = h.synchronize()
        torch.cuda.synchronize()
        assert torch.isfinite(C).all()
        assert (y - ref).abs().max().item() / ref.abs().max().item() < 2e-5
        torch.testing.assert_close(y.sum(1), torch.ones(M, device=dev), atol=1e-4, rtol=0)
    y2 = ops.gemm_nt_softmax(A, B, bias, ops.BIAS_COL, axis=1)      # counters / flags left clean
    torch.testing.assert_close(y2, y, atol=1e-6, rtol=1e-5)
