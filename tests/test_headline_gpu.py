"""GPU numerics at the HEADLINE geometry (BASELINE.json: FF AmazonCat-14k 597540-1000-14588, batch 1000;
conv2d 100 x 3x112x112, 64 filters 7x7): the exact kernels, configs and split-K factors bench.py runs,
compared against plain fp32 PyTorch references (sampled rows where a full fp32 reference is large).

Reference drivers: src/tests/source/FFTestWithDeduplication.cc:353 (load_independent_FF_sets 50, 10000,
1000, 597540, 1000, 14588) and src/tests/source/PipelinedConv2dMemFuseTest.cc."""
import tempfile

import pytest
import torch

from netsdb_amd import _ext, ops

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
K1 = 597568          # 597540 features padded to a multiple of 8 (16-B rows for the LDS-DMA)


def _err(x, ref):
    return (x.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-12)


@pytest.fixture(scope="module")
def layer1_operands():
    g = torch.Generator(device=DEV).manual_seed(11)
    A = torch.empty(1000, K1, device=DEV).uniform_(-1, 1, generator=g).to(torch.bfloat16)
    B = torch.empty(1000, K1, device=DEV).uniform_(-1, 1, generator=g).to(torch.bfloat16)
    rows = torch.randperm(1000, generator=torch.Generator().manual_seed(3))[:32].to(DEV)
    rows[0] = 999                     # last row of the ragged 4th 256-row tile
    ref = A[rows].float() @ B.float().t()
    yield A, B, rows, ref
    del A, B


def test_layer1_auto_config_is_splitk16_8phase(layer1_operands):
    """The launcher's own choice at the headline shape: 16 split-K slices of the 8-phase 256^2 kernel."""
    assert ops.gemm_splits(1000, 1000, K1) == 16


@pytest.mark.parametrize("splits", [0, 16, 17, 24])
def test_layer1_gemm_vs_fp32(layer1_operands, splits):
    """splits 0 = auto (16: the reducer's 16-deep preload), 17 / 24 = the reducer's >16 tail loop."""
    A, B, rows, ref = layer1_operands
    C = ops.gemm_nt(A, B, out_dtype=torch.float32, splits=splits)
    assert C.shape == (1000, 1000)
    e = _err(C[rows], ref)
    assert e < 1e-4, f"splits={splits}: rel err {e}"


def test_layer1_fused_epilogue_bf16_padded_ldc(layer1_operands):
    """The bench's layer-1 call: bias per column + relu, bf16 out into a 64-padded row (ldc 1024)."""
    A, B, rows, ref = layer1_operands
    bias = torch.randn(1000, device=DEV) * 50
    out = torch.empty(1000, 1024, dtype=torch.bfloat16, device=DEV)[:, :1000]
    ops.gemm_nt(A, B, bias, ops.BIAS_COL, ops.ACT_RELU, out_dtype=torch.bfloat16, out=out)
    e = _err(out[rows], torch.relu(ref + bias))
    assert e < 8e-3, e


@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_layer2_gemm_padded_ldc_vs_fp32(out_dtype):
    """FF output layer 1000 x 14588 x 1000 (no split, 8-phase) with bias + exp into a 64-padded ldc."""
    g = torch.Generator(device=DEV).manual_seed(12)
    A = (torch.empty(1000, 1000, device=DEV).uniform_(-1, 1, generator=g) * 0.05).to(torch.bfloat16)
    B = (torch.empty(14588, 1000, device=DEV).uniform_(-1, 1, generator=g) * 0.05).to(torch.bfloat16)
    bias = torch.empty(14588, device=DEV).uniform_(-0.1, 0.1, generator=g)
    assert ops.gemm_splits(1000, 14588, 1000) == 1
    out = torch.empty(1000, 14592, dtype=out_dtype, device=DEV)[:, :14588]
    ops.gemm_nt(A, B, bias, ops.BIAS_COL, ops.ACT_EXP, out_dtype=out_dtype, out=out)
    ref = torch.exp(A.float() @ B.float().t() + bias)
    e = _err(out, ref)
    assert e < (1e-5 if out_dtype == torch.float32 else 8e-3), e


def test_ff_inference_unit_headline_vs_fp32():
    """ff.inference_unit at 597540-1000-14588 through the engine (fused plan, dropout 0) vs the fp32
    network on 32 sampled batch rows (the hidden activations rounded to bf16 as the plan stores them)."""
    from netsdb_amd.client import PDBClient
    from netsdb_amd.models import ff
    from netsdb_amd.models.blocks import to_tensor

    c = PDBClient(root=tempfile.mkdtemp(), device=DEV)
    ff.load_model(c, "ff", 1000, 597540, 1000, 14588, 50, 10000, seed=1234)
    res = ff.inference_unit(c, "ff", "w1", "wo", "inputs", "b1", "bo", "output", dropout_rate=0.0)
    fused = [op for j in res["jobs"] for op in j.get("fused_ops", [])]
    assert any(op.startswith("matmul") for op in fused) and any(op.startswith("softmax") for op in fused)
    out = to_tensor(c, "ff", "output").float()
    assert out.shape == (1000, 14588)
    rows = torch.randperm(1000, generator=torch.Generator().manual_seed(5))[:32].to(DEV)
    x = to_tensor(c, "ff", "inputs")[rows].float()
    w1, b1 = to_tensor(c, "ff", "w1").float(), to_tensor(c, "ff", "b1").float().reshape(-1)
    wo, bo = to_tensor(c, "ff", "wo").float(), to_tensor(c, "ff", "bo").float().reshape(-1)
    y = torch.relu(x @ w1.t() + b1).to(torch.bfloat16).float()          # [32, hidden]
    ref = torch.softmax(y @ wo.t() + bo, dim=-1)
    e = _err(out[rows], ref)
    assert e < 1e-3, e
    assert torch.allclose(out[rows].sum(-1), torch.ones(32, device=DEV), atol=1e-3)
    # the in-kernel operand prefetch changes nothing in the result: the same job without it is bit-identical
    c.engine.operand_prefetch = False
    ff.inference_unit(c, "ff", "w1", "wo", "inputs", "b1", "bo", "output", dropout_rate=0.0)
    torch.testing.assert_close(to_tensor(c, "ff", "output").float(), out, rtol=0, atol=0)


def test_conv2d_headline_vs_fp32():
    """The bench's conv job: 100 images 3x112x112, 64 filters 7x7, stride 1, no padding, vs F.conv2d fp32."""
    from netsdb_amd.client import PDBClient
    from netsdb_amd.models import conv2d as cv

    c = PDBClient(root=tempfile.mkdtemp(), device=DEV)
    c.create_database("conv2d")
    cv.load_images(c, "conv2d", "img", 100, 3, 112, 112, seed=99)
    w, b = cv.random_kernel(64, 3, 7, 7, seed=7, device=DEV)
    cv.conv2d_memfuse_inference(c, "conv2d", "img", "conv_out", w, b)
    x = c.storage.get_set("conv2d", "img").all().columns["data"]
    y = c.storage.get_set("conv2d", "conv_out").all().columns["data"]
    assert tuple(y.shape) == (100, 64, 106, 106)
    wb = w.to(torch.bfloat16).float()
    ref = torch.nn.functional.conv2d(x.float(), wb, b.float())
    e = _err(y, ref)
    assert e < 8e-3, e


def test_native_hip_extension_loaded():
    """The GEMM/conv entry points resolve to the in-tree HIP extension (no eager fallback on a GPU)."""
    mod = _ext.hip()
    assert hasattr(mod, "gemm_nt") and hasattr(mod, "conv2d")
    assert "netsdb_amd" in getattr(mod, "__file__", "")
