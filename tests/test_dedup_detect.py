"""Accuracy-guarded approximate deduplication detector (models/dedup_detect.py; reference
model-inference/deduplication/indexing: blocker.py, indexer.py, lsh/l2lsh.py, deduplicator.py)."""
import pytest
import torch

from netsdb_amd.models import dedup_detect as dd


def _model(g, shapes):
    return [torch.randn(*s, generator=g) * 0.1 for s in shapes]


def test_block_model_roundtrip_and_magnitudes():
    g = torch.Generator().manual_seed(0)
    ws = _model(g, [(37, 20), (20,), (20, 9)])
    st = dd.block_model(ws, 8, 5)
    assert st.block_num == [(5, 4), (3, 1), (3, 2)]
    for a, b in zip(dd.reconstruct(st), ws):
        assert torch.equal(a, b)
    assert st.real_extent((0, 4, 3)) == (5, 5) and st.is_padded((0, 4, 3)) and not st.is_padded((0, 0, 0))
    assert st.real_extent((1, 2, 0)) == (4, 1) and st.is_padded((1, 0, 0))
    # dedup_by_layer: the largest layer's blocks sort first; magnitude of an interior block = its normalised q3
    order = [k for k, _ in sorted(st.magnitude.items(), key=lambda kv: kv[1])]
    assert all(k[0] == 0 for k in order[:20])
    w0 = ws[0]
    blk = w0[8:16, 5:10]
    q3 = torch.quantile(blk.reshape(-1), 0.75).item()
    expect = (q3 - w0.min().item()) / (w0.max().item() - w0.min().item()) - 37 * 20
    assert abs(st.magnitude[(0, 1, 1)] - expect) < 1e-6


def _planted(g, device="cpu", dtype=torch.float32):
    m1 = _model(g, [(64, 48), (48, 16)])
    m2 = [w.clone() for w in _model(g, [(64, 48), (48, 16)])]
    planted = {(0, 1, 2): (0, 3, 0), (0, 2, 1): (0, 0, 1), (1, 1, 0): (1, 2, 1)}   # m2 block <- m1 block
    for (w2, i2, j2), (w1, i1, j1) in planted.items():
        src = m1[w1][i1 * 16:(i1 + 1) * 16, j1 * 8:(j1 + 1) * 8]
        m2[w2][i2 * 16:(i2 + 1) * 16, j2 * 8:(j2 + 1) * 8] = src + torch.rand(src.shape, generator=g) * 0.004
    ix = dd.BlockIndexer(16, 8, device=device, dtype=dtype)
    ix.build_index(dd.block_model([w.to(device, dtype) for w in m1], 16, 8), "m1")
    st2 = dd.block_model([w.to(device, dtype) for w in m2], 16, 8)
    return ix, st2, planted


@pytest.mark.parametrize("use_lsh", [False, True])
def test_dedup_finds_planted_near_duplicates(use_lsh):
    g = torch.Generator().manual_seed(1)
    ix, st2, planted = _planted(g)
    lsh = None
    if use_lsh:
        lsh = dd.L2LSH(16 * 8, r=0.5, num_k=1, num_l=16, seed=0)
        lsh.insert(ix.blocks)
    rep = dd.deduplicate_model(st2, ix, fp=0.01, sim=0.9, use_lsh=use_lsh, lsh=lsh)
    got = {r["duplicate_block_idx"]: ix.ids[r["deduplicate_block_idx"]][1:] for r in rep if r["is_deduplicated"]}
    assert got == planted
    assert len(rep) == len(st2.keys()) and dd.dedup_summary(rep)["deduplicated"] == 3
    for k, src in planted.items():                       # the replaced blocks now hold the indexed block
        assert torch.equal(st2.block(k), ix.blocks[[i for i, t in enumerate(ix.ids) if t[1:] == src][0]])


def test_dedup_accuracy_guard_restores_past_budget():
    """Accuracy = 1 - 0.01 per replaced block, budget 0.025. Evaluating after every replacement keeps 2;
    eval_step 3 (deduplicator.py's step counting: evaluations at replacements 2, 4, ...) also keeps 2 (the
    over-budget 4th evaluation restores replacements 3 and 4); eval_step 4 first evaluates at replacement 3,
    over budget with no earlier in-budget evaluation, and restores every replaced block."""
    for eval_step, keep in ((1, 2), (3, 2), (4, 0)):
        g = torch.Generator().manual_seed(2)
        m = _model(g, [(64, 48)])
        ix = dd.BlockIndexer(16, 8)
        ix.build_index(dd.block_model(m, 16, 8), "m")
        # a copy of the same model: every block has an exact match (its own), excluded via self_index except for
        # a near-duplicate twin planted in every block position of a second indexed model
        twin = [w + 0.001 for w in m]
        finder = ix.build_index(dd.block_model(twin, 16, 8), "twin")
        st = dd.block_model([w.clone() for w in m], 16, 8)
        orig = [w.clone() for w in dd.reconstruct(st)]

        def evaluate(ws):
            return 1.0 - 0.01 * sum(int(not torch.equal(a[i * 16:(i + 1) * 16, j * 8:(j + 1) * 8],
                                                        b[i * 16:(i + 1) * 16, j * 8:(j + 1) * 8]))
                                    for a, b in zip(ws, orig) for i in range(4) for j in range(6))

        own = {k: v - 24 for k, v in finder.items()}      # the first model's pool ids
        rep = dd.deduplicate_model(st, ix, evaluate=evaluate, fp=0.01, sim=0.9, stop_acc_drop=0.025,
                                   eval_step=eval_step, self_index=own)
        kept = sum(r["is_deduplicated"] for r in rep)
        assert kept == keep, (eval_step, kept)
        assert 1.0 - evaluate(dd.reconstruct(st)) <= 0.025 + 1e-9
        assert abs(evaluate(dd.reconstruct(st)) - (1.0 - 0.01 * keep)) < 1e-9


def test_indexer_save_load(tmp_path):
    g = torch.Generator().manual_seed(3)
    ix = dd.BlockIndexer(16, 8)
    ix.build_index(dd.block_model(_model(g, [(40, 20)]), 16, 8), "a")
    p = str(tmp_path / "ix.safetensors")
    ix.save(p)
    ix2 = dd.BlockIndexer.load(p)
    assert torch.equal(ix2.blocks, ix.blocks) and ix2.ids == ix.ids and ix2.model_names == {"a"}


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_block_simcount_kernel_vs_cpu(dtype):
    g = torch.Generator().manual_seed(4)
    pool = (torch.randn(40, 16, 24, generator=g) * 0.02).to(dtype)
    q = pool[7].clone()
    q[3:, 5:] += 0.5 * torch.rand(13, 19, generator=g).to(dtype)
    cand = torch.tensor([7, 0, 39, 12, 7], dtype=torch.int64)
    for h, w in ((16, 24), (11, 17), (16, 1)):
        ref = dd.similarity(pool, cand, q, h, w, 0.01)
        got = dd.similarity(pool.cuda(), cand.cuda(), q.cuda(), h, w, 0.01).cpu()
        assert torch.allclose(got, ref), (h, w, got, ref)


@pytest.mark.gpu
def test_dedup_detector_gpu_matches_cpu():
    g = torch.Generator().manual_seed(1)
    ix, st2, planted = _planted(g, device="cuda:0", dtype=torch.bfloat16)
    rep = dd.deduplicate_model(st2, ix, fp=0.01, sim=0.9)
    got = {r["duplicate_block_idx"]: ix.ids[r["deduplicate_block_idx"]][1:] for r in rep if r["is_deduplicated"]}
    assert got == planted
