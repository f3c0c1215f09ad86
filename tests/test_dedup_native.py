"""Dedup kernels (csrc/kernels/dedup.hip) vs the canonical torch reference, SharedInference vs per-model
fp32 GEMMs, and the config-5 harness (scripts/bench_dedup.py) end to end at a small geometry."""
import json
import os
import subprocess
import sys

import pytest
import torch

from netsdb_amd.models import dedup

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shared_inference_matches_per_model():
    g = torch.Generator().manual_seed(3)
    base = torch.randn(24, 120, generator=g)
    pool = dedup.BlockPool(8, 20, dtype=torch.float32)
    models = {}
    for i in range(4):
        m = base.clone()
        m[:, 100:] = torch.randn(24, 20, generator=g)           # private last column block
        models[f"m{i}"] = m
        pool.add_model(f"m{i}", m)
    si = dedup.SharedInference(pool.index.tables, pool.index.shapes,
                               lambda ids: pool.blocks.index_select(0, ids.to(pool.blocks.device)), 8, 20)
    assert si.common_cols.numel() == 5 and si.priv_cols.numel() == 1
    X = torch.randn(7, 120, generator=g)
    got = si.run(X)
    for n, m in models.items():
        torch.testing.assert_close(got[n], m @ X.t(), rtol=1e-4, atol=1e-4)


def test_bench_dedup_json_line():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "bench_dedup.py"), "--rows", "20", "--cols",
                          "4000", "--block-rows", "10", "--block-cols", "400", "--shared-blocks", "9", "--models", "3",
                          "--steps", "1", "--warmup", "1"], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["blocks_in"] == 60 and line["blocks_stored"] == 18 + 2 * 3
    assert line["rel_err_model0"] < 1e-3 and line["value"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,shape", [(torch.bfloat16, (37, 100, 10000)), (torch.float32, (5, 64, 64)),
                                         (torch.bfloat16, (3000, 8, 16))])
def test_block_hash_kernel_matches_reference(dtype, shape):
    from netsdb_amd import _ext

    assert hasattr(_ext.hip(), "block_hash_partial")
    b = torch.randn(*shape, device="cuda:0").to(dtype)
    b[1] = b[0]
    h = dedup.block_hashes(b)
    assert torch.equal(h, dedup.block_hashes_reference(b))
    assert h[0] == h[1] and h.unique().numel() == shape[0] - 1


@pytest.mark.gpu
def test_block_maxdiff_kernel_and_pool_on_gpu():
    pool = torch.randn(50, 100, 1000, device="cuda:0").to(torch.bfloat16)
    cand = torch.tensor([3, 7, 49, 0], device="cuda:0")
    blks = pool[cand].clone()
    blks[2, 5, 7] += 1.0
    d = dedup.block_maxdiff(pool, cand, blks)
    ref = (pool[cand].float() - blks.float()).abs().flatten(1).amax(1)
    assert torch.equal(d, ref) and d[2] > 0 and d[0] == 0
    bp = dedup.BlockPool(100, 1000, device="cuda:0")
    m = torch.randn(400, 5000, device="cuda:0")
    bp.add_model("a", m)
    m2 = m.clone()
    m2[:100, :1000] += 1
    bp.add_model("b", m2)
    assert bp.stats["blocks_stored"] == 21
    torch.testing.assert_close(bp.materialize("b").float(), m2.to(torch.bfloat16).float())
