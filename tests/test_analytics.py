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
