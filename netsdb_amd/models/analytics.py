"""Analytics libraries on the netsDB computation model — k-means, Gaussian mixture EM, PageRank and LDA
(reference: src/sharedLibraries/headers/KMeans*.h (KMeansQuery, KMeansAggregate, KMeansSampleSelection,
KMeansNormVectorMap, KMeansDataCountAggregate), GMM/Gmm*.h (GmmModel, GmmAggregateLazy,
GmmSampleSelection, GmmDataCountAggregate), URLURLsRank.h / JoinRankedUrlWithLink.h /
URLRankMultiSelection.h / RankUpdateAggregation.h (+ tests/source/PageRank.cc), LDA/*.h).

MI355X-first formulation: every per-record UDF is vectorised over a whole record batch, so the
hot loops are tensor ops on the set's device:

* k-means assignment = one distance GEMM  ``|x|^2 - 2 X C^T + |c|^2`` + argmin per batch, the
  centroid update an AggregateComp keyed by cluster over ``[x, 1]`` value rows (device index_add);
* GMM E-step = batched Cholesky solves for every component; the M-step statistics
  (sum r, sum r x, sum r x x^T) are produced per batch by a MultiSelectionComp as ONE partial
  record per component (two GEMMs ``R^T X`` and ``X^T diag(r_k) X``) and combined by an
  AggregateComp keyed by component — the reference's "lazy" GMM aggregate;
* PageRank = ranks ⋈ out-degree ⋈ edges -> contribution per destination -> AggregateComp sum;
* LDA = documents ⋈ doc-topic ⋈ word-topic -> per-(doc, word) topic assignment sampling
  (``torch.multinomial`` over the collapsed conditional) -> two aggregates rebuild the counts.
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import ops

from ..computations import AggregateComp, JoinComp, MultiSelectionComp, ScanSet, SelectionComp, WriteSet
from ..lambdas import make_batch_lambda, make_lambda_from_member, make_lambda_from_self
from ..objects.builtin import DoubleVector
from ..objects.record import PDBObject, RecordBatch, Tensor
from ..utils.sampler import fraction_for_sample_size, randomize_in_place


def _dev(b: RecordBatch):
    return b.device   # tensor, string and nested columns all count


def _run_to_batch(client, db: str, out: str, comp, job: str) -> Optional[RecordBatch]:
    if client.storage.has_set(db, out):
        client.remove_set(db, out)
    client.create_set(db, out, None)
    client.execute_computations(WriteSet(db, out).set_input(comp), job_name=job)
    got = [b for b in client.get_set_batches(db, out, gather=True) if b.n]
    if not got:
        return None
    b = RecordBatch.concat(got)
    if len(b.columns) == 1:
        v = next(iter(b.columns.values()))
        if isinstance(v, RecordBatch):
            return v
    return b


def load_vectors(client, db: str, name: str, X: torch.Tensor):
    """Store rows of ``X`` as DoubleVector records (ScanKMeansDoubleVectorSet / WriteKMeansSet)."""
    client.create_database(db)
    client.create_set(db, name, DoubleVector)
    client.send_data(db, name, RecordBatch({"data": X}, X.shape[0], DoubleVector))


class _KeyedSum(AggregateComp):
    """Vectorised AggregateComp: key column + [n, F] value rows summed per key."""

    def __init__(self, key_fn, val_fn):
        super().__init__()
        self.key_fn, self.val_fn = key_fn, val_fn

    def get_key_projection(self, x):
        return make_batch_lambda(x, self.key_fn)

    def get_value_projection(self, x):
        return make_batch_lambda(x, self.val_fn)

    def make_output(self, keys, values):
        return RecordBatch({"key": keys, "value": values}, len(values))


# ---------------------------------------------------------------------------------------- k-means
def _sq_dists(X: torch.Tensor, C: torch.Tensor) -> torch.Tensor:
    """|x - c|^2 for all pairs via one GEMM (the norm expansion of KMeansNormVectorMap): -2 X.C^T runs on the
    exact-f32 MFMA kernel on the GPU (ops.gemm_nt_f32), in the data's dtype on the CPU."""
    C = C.to(X.device, X.dtype)
    xc = ops.gemm_nt_f32(X, C, alpha=-2.0)
    return (X * X).sum(1, keepdim=True).to(xc.dtype) + xc + (C * C).sum(1).unsqueeze(0).to(xc.dtype)


class KMeansSampleSelection(SelectionComp):
    """Bernoulli sample of the data for centroid initialisation (reference KMeansSampleSelection)."""

    def __init__(self, fraction: float, seed: int = 0):
        super().__init__()
        self.fraction, self.seed = fraction, seed

    def get_selection(self, x):
        def pick(b):
            g = torch.Generator().manual_seed(self.seed + b.n)
            return (torch.rand(b.n, generator=g) < self.fraction).to(_dev(b))

        return make_batch_lambda(x, pick)

    def get_projection(self, x):
        return make_lambda_from_self(x)


class KMeansAggregate(AggregateComp):
    """key = index of the closest centroid, value = [x, 1]; output = new centroid sums and counts."""

    def __init__(self, centroids: torch.Tensor):
        super().__init__()
        self.centroids = centroids

    def get_key_projection(self, x):
        return make_batch_lambda(x, lambda b: _sq_dists(b.columns["data"], self.centroids).argmin(1))

    def get_value_projection(self, x):
        def val(b):
            X = b.columns["data"]
            return torch.cat([X, torch.ones(X.shape[0], 1, dtype=X.dtype, device=X.device)], 1)

        return make_batch_lambda(x, val)

    def make_output(self, keys, values):
        return RecordBatch({"cluster": keys, "sum": values[:, :-1], "count": values[:, -1]}, len(values))


def kmeans(client, db: str, name: str, k: int, iters: int = 10, init: Optional[torch.Tensor] = None,
           seed: int = 0, tol: float = 0.0):
    """Lloyd iterations (KMeansQuery): returns (centroids [k, d], per-iteration shift list)."""
    if init is None:
        # sample size as the reference driver: Sampler::computeFractionForSampleSize(k, total, false)
        total = sum(b.n for b in client.get_set_batches(db, name))
        total = int(client.ctx.all_reduce_scalar(float(total), "sum")) if client.ctx.distributed else total
        frac = fraction_for_sample_size(k, total, with_replacement=False)
        s = _run_to_batch(client, db, f"{name}_kmeans_sample",
                          KMeansSampleSelection(frac, seed).set_input(ScanSet(db, name, DoubleVector)), "kmeans_sample")
        pts = s.columns["data"] if s is not None and s.n >= k else None
        if pts is None:
            pts = RecordBatch.concat(client.get_set_batches(db, name, gather=True)).columns["data"]
        pts = randomize_in_place(pts.clone(), torch.Generator().manual_seed(seed))
        init = pts[:k].clone()
    C = init.clone()
    shifts = []
    for it in range(iters):
        agg = KMeansAggregate(C).set_input(ScanSet(db, name, DoubleVector))
        r = _run_to_batch(client, db, f"{name}_kmeans_agg", agg, f"kmeans_iter{it}")
        newC = C.clone()
        cl = r.columns["cluster"].long().to(C.device)
        cnt = r.columns["count"].to(C.device, C.dtype).unsqueeze(1)
        newC[cl] = r.columns["sum"].to(C.device, C.dtype) / cnt
        shift = float((newC - C).norm())
        shifts.append(shift)
        C = newC
        if shift <= tol:
            break
    return C, shifts


def kmeans_reference(X: torch.Tensor, init: torch.Tensor, iters: int):
    C = init.clone().double()
    X = X.double()
    for _ in range(iters):
        a = _sq_dists(X, C).argmin(1)
        for j in range(C.shape[0]):
            m = a == j
            if m.any():
                C[j] = X[m].mean(0)
    return C


# ------------------------------------------------------------------------------------------- GMM
class GmmModel:
    """weights [k], means [k, d], covars [k, d, d]; Cholesky factors and log-determinants cached
    (reference GmmModel::calcInvCovars via gsl Cholesky)."""

    def __init__(self, weights, means, covars):
        self.weights, self.means, self.covars = weights, means, covars
        self.update()

    def update(self):
        self.chol = torch.linalg.cholesky(self.covars)
        self.logdet = 2.0 * torch.log(torch.diagonal(self.chol, dim1=-2, dim2=-1)).sum(-1)
        # whitening L^-1 per component: Mahalanobis terms of all components become ONE GEMM per batch
        eye = torch.eye(self.chol.shape[-1], dtype=self.chol.dtype, device=self.chol.device)
        self.chol_inv = torch.linalg.solve_triangular(self.chol, eye.expand_as(self.chol), upper=False)

    def log_resp(self, X: torch.Tensor):
        """log(w_k N(x | mu_k, S_k)) for every row and component, and the row log-likelihood.
        z_k = L_k^-1 (x - mu_k) for every component at once: [k*d, d] x X^T on the matrix cores (ops.gemm_nt_f32)
        minus L_k^-1 mu_k."""
        d = X.shape[1]
        k = self.means.shape[0]
        dev, dt = X.device, X.dtype
        Li = self.chol_inv.to(dev, dt)                                                  # [k, d, d]
        z = ops.gemm_nt_f32(Li.reshape(k * d, d), X).to(dt).reshape(k, d, -1)          # [k, d, n]
        z = z - torch.bmm(Li, self.means.to(dev, dt).unsqueeze(2))                      # - L^-1 mu
        maha = (z * z).sum(1)                                                           # [k, n]
        lp = (torch.log(self.weights.to(dev, dt)).unsqueeze(1) - 0.5 * (d * torch.log(torch.tensor(2 * torch.pi, dtype=dt))
                                                                        + self.logdet.to(dev, dt).unsqueeze(1) + maha))
        ll = torch.logsumexp(lp, 0)
        return lp - ll.unsqueeze(0), ll


class GmmStats(PDBObject):
    comp: int
    stats: Tensor()


class GmmPartialStats(MultiSelectionComp):
    """One partial-statistics record per component per input batch: [sum r, sum r x, sum r x x^T, ll]."""

    def __init__(self, model: GmmModel):
        super().__init__()
        self.model = model

    def get_selection(self, x):
        return make_batch_lambda(x, lambda b: torch.ones(b.n, dtype=torch.bool, device=_dev(b)))

    def get_projection(self, x):
        def proj(b):
            X = b.columns["data"]
            lr, ll = self.model.log_resp(X)
            R = lr.exp()                                                   # [k, n]
            k, d = R.shape[0], X.shape[1]
            s0 = R.sum(1, keepdim=True)                                    # [k, 1]
            Xt = X.t().contiguous()                                        # [d, n]: K = n contiguous
            s1 = ops.gemm_nt_f32(R, Xt).to(X.dtype)                        # [k, d] = R . X
            # second moments sum_n r_kn x_n x_n^T: (r_k * X^T) . X as one [k*d, n] x [d, n]^T GEMM
            s2 = ops.gemm_nt_f32((R.unsqueeze(1) * Xt.unsqueeze(0)).reshape(k * d, -1), Xt).to(X.dtype)
            s2 = s2.reshape(k, d * d)                                      # [k, d*d]
            llc = torch.zeros(k, 1, dtype=X.dtype, device=X.device)
            llc[0, 0] = ll.sum()
            return RecordBatch({"comp": torch.arange(k, device=X.device), "stats": torch.cat([s0, s1, s2, llc], 1)}, k,
                               GmmStats)

        return make_batch_lambda(x, proj)


def gmm(client, db: str, name: str, k: int, iters: int = 10, init_means: Optional[torch.Tensor] = None,
        reg: float = 1e-6):
    """EM for a full-covariance Gaussian mixture; returns (model, log-likelihood per iteration)."""
    data = RecordBatch.concat(client.get_set_batches(db, name, gather=True)).columns["data"]
    d = data.shape[1]
    dt = data.dtype
    # model parameters (k x d x d) live on the host; log_resp / the stats UDF move them to the set's device
    means = (init_means if init_means is not None else data[:k]).detach().cpu().clone().to(dt)
    cov0 = torch.cov(data.T.double()).cpu().to(dt) + reg * torch.eye(d, dtype=dt)
    model = GmmModel(torch.full((k,), 1.0 / k, dtype=dt), means, cov0.unsqueeze(0).repeat(k, 1, 1).clone())
    lls = []
    for it in range(iters):
        part = GmmPartialStats(model).set_input(ScanSet(db, name, DoubleVector))
        agg = _KeyedSum(lambda b: b.columns["comp"], lambda b: b.columns["stats"]).set_input(part)
        r = _run_to_batch(client, db, f"{name}_gmm_stats", agg, f"gmm_iter{it}")
        order = torch.argsort(r.columns["key"].cpu())
        S = r.columns["value"].cpu()[order]
        s0, s1, s2 = S[:, 0], S[:, 1:1 + d], S[:, 1 + d:1 + d + d * d].reshape(k, d, d)
        lls.append(float(S[:, -1].sum()))
        n = s0.sum()
        mu = s1 / s0.unsqueeze(1)
        cov = s2 / s0.view(k, 1, 1) - mu.unsqueeze(2) * mu.unsqueeze(1) + reg * torch.eye(d, dtype=dt)
        model = GmmModel(s0 / n, mu, cov)
    return model, lls


def gmm_reference(X: torch.Tensor, k: int, iters: int, init_means: torch.Tensor, reg: float = 1e-6):
    X = X.double()
    d = X.shape[1]
    cov0 = torch.cov(X.T) + reg * torch.eye(d, dtype=torch.float64)
    model = GmmModel(torch.full((k,), 1.0 / k, dtype=torch.float64), init_means.double().clone(),
                     cov0.unsqueeze(0).repeat(k, 1, 1).clone())
    lls = []
    for _ in range(iters):
        lr, ll = model.log_resp(X)
        lls.append(float(ll.sum()))
        R = lr.exp()
        s0 = R.sum(1)
        mu = (R @ X) / s0.unsqueeze(1)
        cov = torch.einsum("kn,ni,nj->kij", R, X, X) / s0.view(k, 1, 1) - mu.unsqueeze(2) * mu.unsqueeze(1) + \
            reg * torch.eye(d, dtype=torch.float64)
        model = GmmModel(s0 / X.shape[0], mu, cov)
    return model, lls


# -------------------------------------------------------------------------------------- PageRank
class Edge(PDBObject):
    src: int
    dst: int


class RankedUrl(PDBObject):
    url: int
    rank: float


class _EdgeJoin(JoinComp):
    """(ranks ⋈ out-degree) ⋈ edges on src: contribution rank/deg to every destination
    (JoinRankedUrlWithLink + URLRankMultiSelection, edge-list form)."""

    def __init__(self):
        super().__init__(3)

    def get_selection(self, r, deg, e):
        return (make_lambda_from_member(r, "url") == make_lambda_from_member(deg, "key")) & \
            (make_lambda_from_member(r, "url") == make_lambda_from_member(e, "src"))

    def get_projection(self, r, deg, e):
        def proj(rb, db_, eb):
            return RecordBatch({"dst": eb.columns["dst"],
                                "contrib": rb.columns["rank"].double() / db_.columns["value"][:, 0].double()}, eb.n)

        return make_batch_lambda(r, deg, e, proj)


class RankUpdateAggregation(AggregateComp):
    def __init__(self, damping: Optional[float], n: int):
        super().__init__()
        self.damping, self.n = damping, n

    def get_key_projection(self, x):
        return make_lambda_from_member(x, "dst")

    def get_value_projection(self, x):
        return make_lambda_from_member(x, "contrib")

    def make_output(self, keys, values):
        v = values.double()
        if self.damping is not None:
            v = (1.0 - self.damping) / self.n + self.damping * v
        return RecordBatch({"url": keys, "rank": v}, len(values), RankedUrl)


def load_graph(client, db: str, src: torch.Tensor, dst: torch.Tensor, n: int):
    client.create_database(db)
    client.create_set(db, "links", Edge)
    client.send_data(db, "links", RecordBatch({"src": src.long(), "dst": dst.long()}, src.numel(), Edge))
    client.create_set(db, "rankings_0", RankedUrl)
    client.send_data(db, "rankings_0", RecordBatch({"url": torch.arange(n), "rank": torch.full((n,), 1.0 / n,
                                                                                              dtype=torch.float64)},
                                                   n, RankedUrl))


def pagerank(client, db: str, n: int, iters: int = 10, damping: Optional[float] = 0.85) -> torch.Tensor:
    """Iterative ranks (tests/source/PageRank.cc). ``damping=None`` is the reference's undamped update."""
    deg = _KeyedSum(lambda b: b.columns["src"], lambda b: torch.ones(b.n, 1, dtype=torch.float64, device=_dev(b)))
    if not client.storage.has_set(db, "outdeg"):
        client.create_set(db, "outdeg", None)
        client.execute_computations(WriteSet(db, "outdeg").set_input(deg.set_input(ScanSet(db, "links", Edge))),
                                    job_name="pagerank_outdeg")
    cur = "rankings_0"
    for it in range(iters):
        nxt = f"rankings_{1 + it % 2}"            # ping-pong; rankings_0 (the initial ranks) is kept
        j = _EdgeJoin()
        j.set_input(0, ScanSet(db, cur, RankedUrl))
        j.set_input(1, ScanSet(db, "outdeg"))
        j.set_input(2, ScanSet(db, "links", Edge))
        agg = RankUpdateAggregation(damping, n).set_input(j)
        if client.storage.has_set(db, nxt):
            client.remove_set(db, nxt)
        client.create_set(db, nxt, None)
        client.execute_computations(WriteSet(db, nxt).set_input(agg), job_name=f"pagerank_iter{it}")
        cur = nxt
    got = [b for b in client.get_set_batches(db, cur, gather=True) if b.n]
    b = RecordBatch.concat(got)
    if len(b.columns) == 1:
        b = next(iter(b.columns.values()))
    ranks = torch.zeros(n, dtype=torch.float64)
    if damping is not None:
        ranks.fill_((1.0 - damping) / n)       # urls with no in-links keep the teleport mass
    ranks[b.columns["url"].long().cpu()] = b.columns["rank"].double().cpu()
    return ranks


def pagerank_reference(src, dst, n, iters, damping=0.85):
    r = torch.full((n,), 1.0 / n, dtype=torch.float64)
    deg = torch.zeros(n, dtype=torch.float64).index_add_(0, src, torch.ones(src.numel(), dtype=torch.float64))
    for _ in range(iters):
        c = torch.zeros(n, dtype=torch.float64).index_add_(0, dst, r[src] / deg[src])
        if damping is None:
            has = torch.zeros(n, dtype=torch.bool)
            has[dst] = True
            r = torch.where(has, c, torch.zeros_like(c))
        else:
            r = (1 - damping) / n + damping * c
    return r


# ------------------------------------------------------------------------------------------- LDA
class LDADocument(PDBObject):
    doc: int
    word: int
    count: int


class TopicCounts(PDBObject):
    key: int
    value: Tensor()


class LDADocWordTopicJoin(JoinComp):
    """documents ⋈ doc-topic (doc) ⋈ word-topic (word) -> sampled topic counts of every (doc, word)."""

    def __init__(self, alpha: float, beta: float, topic_totals: torch.Tensor, vocab: int, seed: int):
        super().__init__(3)
        self.alpha, self.beta, self.tt, self.V, self.seed = alpha, beta, topic_totals, vocab, seed

    def get_selection(self, d, dt, wt):
        return (make_lambda_from_member(d, "doc") == make_lambda_from_member(dt, "key")) & \
            (make_lambda_from_member(d, "word") == make_lambda_from_member(wt, "key"))

    def get_projection(self, d, dt, wt):
        def proj(db_, dtb, wtb):
            ndk = dtb.columns["value"].double()
            nwk = wtb.columns["value"].double()
            tt = self.tt.to(ndk.device, ndk.dtype)
            p = (ndk + self.alpha) * (nwk + self.beta) / (tt + self.V * self.beta)
            cnt = db_.columns["count"].long()
            g = torch.Generator(device=p.device).manual_seed(self.seed + int(cnt.sum()))
            K = p.shape[1]
            draws = torch.multinomial(p / p.sum(1, keepdim=True), int(cnt.max()) if cnt.numel() else 1,
                                      replacement=True, generator=g)                      # [n, maxc]
            keep = torch.arange(draws.shape[1], device=p.device).unsqueeze(0) < cnt.unsqueeze(1)
            z = torch.zeros(p.shape[0], K, dtype=torch.float64, device=p.device)
            z.scatter_add_(1, draws, keep.double())
            return RecordBatch({"doc": db_.columns["doc"], "word": db_.columns["word"], "z": z}, db_.n)

        return make_batch_lambda(d, dt, wt, proj)


def load_corpus(client, db: str, docs: torch.Tensor, words: torch.Tensor, counts: torch.Tensor):
    client.create_database(db)
    client.create_set(db, "lda_docs", LDADocument)
    client.send_data(db, "lda_docs", RecordBatch({"doc": docs.long(), "word": words.long(), "count": counts.long()},
                                                 docs.numel(), LDADocument))


def lda(client, db: str, n_docs: int, vocab: int, topics: int, iters: int = 10, alpha: float = 0.1,
        beta: float = 0.01, seed: int = 0):
    """Approximate distributed Gibbs LDA; returns (doc-topic [D, K], word-topic [V, K], log-likelihoods)."""
    g = torch.Generator().manual_seed(seed)
    allb = RecordBatch.concat(client.get_set_batches(db, "lda_docs", gather=True))
    docs, words, cnt = (allb.columns[c].long().cpu() for c in ("doc", "word", "count"))
    z0 = torch.zeros(docs.numel(), topics, dtype=torch.float64)
    z0.scatter_add_(1, torch.randint(0, topics, (docs.numel(), 1), generator=g), cnt.double().unsqueeze(1))
    ndk = torch.zeros(n_docs, topics, dtype=torch.float64).index_add_(0, docs, z0)
    nwk = torch.zeros(vocab, topics, dtype=torch.float64).index_add_(0, words, z0)
    lls = []
    for it in range(iters):
        for nm, mat in (("lda_dt", ndk), ("lda_wt", nwk)):
            if client.storage.has_set(db, nm):
                client.remove_set(db, nm)
            client.create_set(db, nm, TopicCounts)
            client.send_data(db, nm, RecordBatch({"key": torch.arange(mat.shape[0]), "value": mat}, mat.shape[0], TopicCounts))
        j = LDADocWordTopicJoin(alpha, beta, nwk.sum(0), vocab, seed + 1000 * it)
        j.set_input(0, ScanSet(db, "lda_docs", LDADocument))
        j.set_input(1, ScanSet(db, "lda_dt", TopicCounts))
        j.set_input(2, ScanSet(db, "lda_wt", TopicCounts))
        if client.storage.has_set(db, "lda_z"):
            client.remove_set(db, "lda_z")
        client.create_set(db, "lda_z", None)
        client.execute_computations(WriteSet(db, "lda_z").set_input(j), job_name=f"lda_sample{it}")
        zb = RecordBatch.concat([b for b in client.get_set_batches(db, "lda_z", gather=True) if b.n])
        if len(zb.columns) == 1:
            zb = next(iter(zb.columns.values()))
        # LDADocTopicAggregate / LDAWordTopicAggregate
        dz = _run_to_batch(client, db, "lda_dt_new", _KeyedSum(lambda b: b.columns["doc"], lambda b: b.columns["z"])
                           .set_input(ScanSet(db, "lda_z")), f"lda_doc_topic{it}")
        wz = _run_to_batch(client, db, "lda_wt_new", _KeyedSum(lambda b: b.columns["word"], lambda b: b.columns["z"])
                           .set_input(ScanSet(db, "lda_z")), f"lda_word_topic{it}")
        ndk = torch.zeros(n_docs, topics, dtype=torch.float64)
        ndk[dz.columns["key"].long().cpu()] = dz.columns["value"].double().cpu()
        nwk = torch.zeros(vocab, topics, dtype=torch.float64)
        nwk[wz.columns["key"].long().cpu()] = wz.columns["value"].double().cpu()
        lls.append(lda_log_likelihood(docs, words, cnt, ndk, nwk, alpha, beta))
    return ndk, nwk, lls


def lda_log_likelihood(docs, words, cnt, ndk, nwk, alpha, beta):
    theta = (ndk + alpha) / (ndk + alpha).sum(1, keepdim=True)
    phi = (nwk + beta) / (nwk + beta).sum(0, keepdim=True)
    p = (theta[docs] * phi[words]).sum(1)
    return float((cnt.double() * torch.log(p)).sum())


__all__ = ["kmeans", "kmeans_reference", "KMeansAggregate", "KMeansSampleSelection", "load_vectors", "gmm",
           "gmm_reference", "GmmModel", "GmmPartialStats", "pagerank", "pagerank_reference", "load_graph", "lda",
           "load_corpus", "LDADocWordTopicJoin", "lda_log_likelihood"]
