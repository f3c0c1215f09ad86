"""FF-NN inference through the engine: fused (MFMA plan) and generic (join/aggregate pipelines)
against a plain fp32 PyTorch reference (reference test: src/tests/source/FFTest.cc)."""
import pytest
import torch

from netsdb_amd.client import PDBClient
from netsdb_amd.models import ff
from netsdb_amd.models.blocks import to_tensor


def _run(tmp_path, fusion, device="cpu", two_layers=False):
    c = PDBClient(root=str(tmp_path), device=device, fusion=fusion)
    batch, feats, hid, labels = 40, 96, 48, 24
    ff.load_model(c, "ff", batch, feats, hid, labels, block_x=16, block_y=32, hidden2=32 if two_layers else None,
                  dtype=torch.float32)
    if two_layers:
        res = ff.inference(c, "ff", "w1", "w2", "wo", "inputs", "b1", "b2", "bo", "output")
    else:
        res = ff.inference_unit(c, "ff", "w1", "wo", "inputs", "b1", "bo", "output")
    c.last_jobs = res["jobs"]
    out = to_tensor(c, "ff", "output")
    g = lambda n: to_tensor(c, "ff", n)  # noqa: E731
    ref = ff.reference_inference(g("inputs"), g("w1"), g("b1"), g("wo"), g("bo"),
                                 g("w2") if two_layers else None, g("b2") if two_layers else None)
    return out.float().cpu(), ref.cpu(), c


@pytest.mark.parametrize("fusion", [True, False])
def test_ff_inference_unit_cpu(tmp_path, fusion):
    out, ref, c = _run(tmp_path, fusion)
    assert out.shape == ref.shape
    torch.testing.assert_close(out, ref, atol=2e-3, rtol=2e-2)
    fused = [op for j in c.last_jobs for op in j.get("fused_ops", [])]
    if fusion:
        # the whole graph lowers onto MFMA GEMMs with fused epilogues: no TCAP pipeline runs
        assert any(op.startswith("matmul[FFTransposeMult") for op in fused), fused
        assert any(op.startswith("epilogue[FFReluBiasSum") for op in fused), fused
        assert any(op.startswith("softmax[FFOutputLayer") for op in fused), fused
        assert c.engine.last_plan is None
    else:
        assert fused == []
        assert c.engine.last_plan is not None and len(c.engine.last_plan.stages) > 0


@pytest.mark.parametrize("fusion", [True, False])
def test_ff_two_hidden_layers_cpu(tmp_path, fusion):
    out, ref, _ = _run(tmp_path, fusion, two_layers=True)
    torch.testing.assert_close(out, ref, atol=2e-3, rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("fusion", [True, False])
def test_ff_inference_unit_gpu(tmp_path, fusion):
    out, ref, _ = _run(tmp_path, fusion, device="cuda:0")
    torch.testing.assert_close(out, ref, atol=1e-2, rtol=5e-2)
