"""k-means / GMM / PageRank / LDA libraries (reference src/sharedLibraries KMeans*, GMM/*, PageRank,
LDA/*) through the engine, checked against plain-torch implementations of the same algorithms."""
import torch

from netsdb_amd.client import PDBClient
from netsdb_amd.models import analytics as A


def _client(tmp_path):
    return PDBClient(root=str(tmp_path), page_size=1 << 14)


def _blobs(n=1500, d=5, k=4, seed=0):
    g = torch.Generator().manual_seed(seed)
    centers = torch.randn(k, d, generator=g, dtype=torch.float64) * 5
    return centers[torch.randint(0, k, (n,), generator=g)] + torch.randn(n, d, generator=g, dtype=torch.float64)


def test_kmeans_matches_lloyd(tmp_path):
    c = _client(tmp_path)
    X = _blobs()
    A.load_vectors(c, "ml", "pts", X)
    init = X[:4].clone()
    C, shifts = A.kmeans(c, "ml", "pts", 4, iters=6, init=init)
    torch.testing.assert_close(C.double(), A.kmeans_reference(X, init, len(shifts)), rtol=1e-5, atol=1e-5)
    # sampled initialisation path (KMeansSampleSelection) runs and converges
    C2, s2 = A.kmeans(c, "ml", "pts", 4, iters=10, seed=3)
    assert C2.shape == (4, 5) and s2[-1] <= s2[0]


def test_gmm_matches_em(tmp_path):
    c = _client(tmp_path)
    X = _blobs(n=1200, d=4, k=3, seed=1)
    A.load_vectors(c, "ml", "pts", X)
    m, lls = A.gmm(c, "ml", "pts", 3, iters=4, init_means=X[:3])
    mr, llr = A.gmm_reference(X, 3, 4, X[:3])
    torch.testing.assert_close(m.means.double(), mr.means, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(m.weights.double(), mr.weights, rtol=1e-4, atol=1e-4)
    assert all(abs(a - b) <= 1e-4 * abs(b) for a, b in zip(lls, llr))
    assert lls[-1] >= lls[0]


def test_pagerank(tmp_path):
    c = _client(tmp_path)
    g = torch.Generator().manual_seed(2)
    n = 150
    src, dst = torch.randint(0, n, (1000,), generator=g), torch.randint(0, n, (1000,), generator=g)
    A.load_graph(c, "g", src, dst, n)
    for damping in (0.85, None):
        r = A.pagerank(c, "g", n, iters=5, damping=damping)
        torch.testing.assert_close(r, A.pagerank_reference(src, dst, n, 5, damping), rtol=1e-9, atol=1e-12)


def test_lda_improves_likelihood(tmp_path):
    c = _client(tmp_path)
    g = torch.Generator().manual_seed(4)
    D, V, K = 40, 60, 3
    docs = torch.arange(D).repeat_interleave(15)
    words = (docs % K) * 20 + torch.randint(0, 20, (D * 15,), generator=g)
    cnts = torch.randint(1, 4, (D * 15,), generator=g)
    A.load_corpus(c, "lda", docs, words, cnts)
    ndk, nwk, ll = A.lda(c, "lda", D, V, K, iters=8)
    assert ndk.sum().item() == cnts.sum().item() == nwk.sum().item()
    assert ll[-1] > ll[0]


# ------------------------------------------------------------------ GPU: the exact-f32 MFMA GEMM behind k-means / GMM
import pytest  # noqa: E402


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(1, 1, 4), (17, 33, 20), (128, 128, 16), (300, 257, 516), (1500, 4, 8), (40, 15, 1200)])
def test_gemm_nt_f32_gpu_vs_fp64(M, N, K):
    from netsdb_amd import ops

    g = torch.Generator(device="cuda:0").manual_seed(M + N + K)
    A_ = torch.randn(M, K, device="cuda:0", generator=g)
    B_ = torch.randn(N, K, device="cuda:0", generator=g)
    C = ops.gemm_nt_f32(A_, B_, alpha=-2.0)
    ref = -2.0 * (A_.double() @ B_.double().t())
    assert C.dtype == torch.float32 and C.shape == (M, N)
    err = ((C.double() - ref).abs().max() / ref.abs().max().clamp(min=1e-30)).item()
    assert err < 2e-6, err                      # f32 products, f32 sums: no bf16 rounding
    acc = torch.ones(M, N, device="cuda:0")
    ops.gemm_nt_f32(A_, B_, out=acc, accumulate=True)
    tol = 2e-6 * (1.0 + ref.abs().max().item())     # the f32 sum with the 1.0 already in C rounds at ~1 ulp of 1
    torch.testing.assert_close(acc.double(), 1.0 + ref / -2.0, rtol=0, atol=tol)


@pytest.mark.gpu
def test_gemm_nt_f32_identity_asymmetric_gpu():
    from netsdb_amd import ops

    n = 64
    A_ = torch.eye(n, device="cuda:0")
    B_ = (torch.arange(n * n, device="cuda:0", dtype=torch.float32).reshape(n, n) % 97) - 48
    torch.testing.assert_close(ops.gemm_nt_f32(A_, B_), B_.t().contiguous(), rtol=0, atol=0)


@pytest.mark.gpu
def test_kmeans_and_gmm_gpu_match_cpu_fp64(tmp_path):
    """k-means and GMM through the engine on the GPU (distance / responsibility GEMMs on the f32 MFMA kernel)
    agree with the fp64 CPU runs of the same library; the GEMM ops issue no host read."""
    from netsdb_amd import ops

    X = _blobs()
    init = X[:4].clone()
    cg = PDBClient(root=str(tmp_path / "g"), page_size=1 << 14, device="cuda:0")
    A.load_vectors(cg, "ml", "pts", X)
    Cg, _ = A.kmeans(cg, "ml", "pts", 4, iters=6, init=init.cuda())
    torch.testing.assert_close(Cg.double().cpu(), A.kmeans_reference(X, init, 6), rtol=1e-5, atol=1e-5)

    Xg = _blobs(n=1200, d=4, k=3, seed=1)
    A.load_vectors(cg, "ml", "gpts", Xg)
    m, lls = A.gmm(cg, "ml", "gpts", 3, iters=4, init_means=Xg[:3].cuda())
    mr, llr = A.gmm_reference(Xg, 3, 4, Xg[:3])
    torch.testing.assert_close(m.means.double().cpu(), mr.means, rtol=1e-4, atol=1e-4)
    assert all(abs(a - b) <= 1e-4 * abs(b) for a, b in zip(lls, llr))

    calls = []
    orig = {k: getattr(torch.Tensor, k) for k in ("cpu", "tolist", "item")}

    def guard(name):
        def w(self, *a, **kw):
            calls.append(name)
            return orig[name](self, *a, **kw)
        return w

    xg = Xg.cuda()
    for k in orig:
        setattr(torch.Tensor, k, guard(k))
    try:
        A._sq_dists(xg, xg[:5])
        m.log_resp(xg)
        ops.gemm_nt_f32(xg, xg)
    finally:
        for k, f in orig.items():
            setattr(torch.Tensor, k, f)
    torch.cuda.synchronize()
    assert calls == [], calls
