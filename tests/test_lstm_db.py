"""LSTM through the database (reference job graph src/tests/source/LSTMTest.cc:165-420): per-gate jobs
lowered onto one MFMA GEMM each (K-concatenated [W | U] . [x ; h], bias matrix + activation in the
epilogue) and the whole step lowered onto one stacked gate GEMM + lstm_cell, vs an fp64 reference."""
import tempfile

import pytest
import torch

from netsdb_amd.client import PDBClient
from netsdb_amd.models import lstm
from netsdb_amd.models.blocks import to_tensor


def _check(device, dims=(400, 500, 128), fusion=True, tol=1e-5):
    D, B, L = dims
    c = PDBClient(root=tempfile.mkdtemp(), device=device, fusion=fusion)
    dt = torch.float32 if device == "cpu" else torch.bfloat16
    lstm.load_lstm_sets(c, "lstm", D, B, L, 100, 100, seed=3, dtype=dt)
    href, cref = lstm.lstm_db_reference(c, "lstm")
    st = lstm.lstm_step_jobs(c, "lstm")
    h1 = to_tensor(c, "lstm", "h_t").double().cpu()
    c1 = to_tensor(c, "lstm", "c_t").double().cpu()
    e = max((h1 - href).abs().max().item(), (c1 - cref).abs().max().item())
    assert e < tol, e
    st2 = lstm.lstm_step_graph(c, "lstm")
    h2 = to_tensor(c, "lstm", "h_t").double().cpu()
    c2 = to_tensor(c, "lstm", "c_t").double().cpu()
    e2 = max((h2 - href).abs().max().item(), (c2 - cref).abs().max().item())
    assert e2 < tol, e2
    return st, st2


@pytest.mark.parametrize("fusion", [True, False])
def test_lstm_job_graph_cpu(fusion):
    st, st2 = _check("cpu", (120, 70, 40), fusion=fusion)
    ops = [op for s in st for op in s.get("fused_ops", [])]
    if fusion:
        assert sum(op.startswith("gate_gemm[") and op.endswith(":2x]") for op in ops) == 4, ops
        assert any(op.startswith("lstm_two_sum") for op in ops) and any(op.startswith("lstm_hidden") for op in ops)
        assert "lstm_step[stacked gate GEMM + lstm_cell]" in st2["fused_ops"]
        assert st2.get("out_of_core", {}).get("lstm_fused_steps") == 1
    else:
        assert ops == []


@pytest.mark.gpu
def test_lstm_job_graph_gpu():
    st, st2 = _check("cuda:0", (400, 500, 128), tol=3e-2)
    assert "lstm_step[stacked gate GEMM + lstm_cell]" in st2["fused_ops"]
