"""Reddit in-database inference pipeline (reference: src/reddit — RedditComment/Author/Sub,
CommentsToFeatures (time + numeric features), CommentChunksToBlocks (features -> matrix blocks by chunk),
CommentBlockToMatrix, the FF inference, CommentInferenceJoin (labels back onto comments),
RedditLabelSelection<i>_<t> / Positive / Negative label selections, ThreeWayJoin (comment ⋈ author ⋈ sub
-> FullFeatures), CommentPartition / AuthorCommentsPartition / SubsCommentsPartition).

Flow (all netsDB computations; the inference is the fused FF plan of :mod:`models.ff`):

  comments --CommentsToFeatures--> features [index, F] --CommentChunksToBlocks--> block rows
  --(DenseMatrixSet "inputs")--> FF inference (GEMM + bias/ReLU epilogue, GEMM + softmax)
  --> InferenceResult(index, label) --CommentInferenceJoin--> labelled comments
  --LabelSelection(threshold)--> positives / negatives;  comments ⋈ authors ⋈ subs -> FullFeatures.

Features are computed vectorised on the batch (UTC timestamps decomposed with integer tensor
arithmetic — the reference's gmtime_r fields: mday, sec, min, hour, mon, year, wday, yday, isdst=0).
"""
from __future__ import annotations

from typing import Dict, List

import torch

from ..computations import AggregateComp, JoinComp, PartitionComp, ScanSet, SelectionComp, WriteSet
from ..lambdas import make_batch_lambda, make_lambda_from_member, make_lambda_from_self
from ..objects.record import PDBObject, RecordBatch, Tensor
from . import blocks as B
from . import ff


class RedditComment(PDBObject):
    index: int
    label: int
    author: str
    subreddit_id: str
    author_created_utc: int
    created_utc: int
    retrieved_on: int
    score: int
    controversiality: int
    gilded: int
    archived: int
    body: str


class RedditAuthor(PDBObject):
    author: str
    comment_karma: int
    link_karma: int
    created_utc: int


class RedditSub(PDBObject):
    name: str
    subscribers: int
    created_utc: int


class CommentFeatures(PDBObject):
    index: int
    features: Tensor()


class InferenceResult(PDBObject):
    index: int
    label: int


class FullFeatures(PDBObject):
    index: int
    author: str
    subreddit: str
    features: Tensor()


TIME_FEATURES = 9


def _time_features(t: torch.Tensor) -> torch.Tensor:
    """gmtime_r fields of UTC seconds, normalised as CommentFeatures.h push_time_features."""
    t = t.long()
    days = torch.div(t, 86400, rounding_mode="floor")
    sod = t - days * 86400
    hour, minute, sec = sod // 3600, (sod % 3600) // 60, sod % 60
    wday = (days + 4) % 7                                   # 1970-01-01 was a Thursday
    # civil-from-days (Howard Hinnant's algorithm), all integer tensor ops
    z = days + 719468
    era = torch.div(z, 146097, rounding_mode="floor")
    doe = z - era * 146097
    yoe = torch.div(doe - doe // 1460 + doe // 36524 - doe // 146096, 365, rounding_mode="floor")
    y = yoe + era * 400
    doy = doe - (365 * yoe + yoe // 4 - yoe // 100)
    mp = (5 * doy + 2) // 153
    mday = doy - (153 * mp + 2) // 5 + 1
    mon = torch.where(mp < 10, mp + 3, mp - 9)              # 1..12
    y = torch.where(mon <= 2, y + 1, y)
    leap = ((y % 4 == 0) & (y % 100 != 0)) | (y % 400 == 0)
    cum = torch.tensor([0, 31, 59, 90, 120, 151, 181, 212, 243, 273, 304, 334], device=t.device)
    yday = cum[mon - 1] + mday - 1 + ((mon > 2) & leap).long()
    tm_year = y - 1900
    f = torch.stack([mday / 31.0, sec / 60.0, minute / 59.0, hour / 23.0, (mon - 1) / 11.0, tm_year / 2021.0,
                     wday / 6.0, yday / 365.0, torch.zeros_like(t, dtype=torch.float64)], 1)
    return f.double()


def comment_features(b: RecordBatch) -> torch.Tensor:
    cols = b.columns
    parts = [_time_features(cols["author_created_utc"]), _time_features(cols["created_utc"]),
             _time_features(cols["retrieved_on"])]
    num = torch.stack([cols[c].double() for c in ("score", "controversiality", "gilded", "archived")], 1)
    parts.append(torch.sign(num) * torch.log1p(num.abs()))
    return torch.cat(parts, 1)


NUM_FEATURES = 3 * TIME_FEATURES + 4


class CommentsToFeatures(SelectionComp):
    def get_selection(self, c):
        return make_batch_lambda(c, lambda b: torch.ones(b.n, dtype=torch.bool, device=b.device))

    def get_projection(self, c):
        return make_batch_lambda(c, lambda b: RecordBatch({"index": b.columns["index"], "features": comment_features(b)},
                                                          b.n, CommentFeatures))


class CommentChunksToBlocks(AggregateComp):
    """key = chunk index (index // chunk_size), value = the chunk's rows scattered into a
    [chunk_size, F] block (sum-combined: every row lands in exactly one slot)."""

    def __init__(self, chunk_size: int):
        super().__init__()
        self.chunk = chunk_size

    def get_key_projection(self, f):
        return make_batch_lambda(f, lambda b: torch.div(b.columns["index"].long(), self.chunk, rounding_mode="floor"))

    def get_value_projection(self, f):
        def val(b):
            x = b.columns["features"]
            blk = torch.zeros(b.n, self.chunk, x.shape[1], dtype=x.dtype, device=x.device)
            blk[torch.arange(b.n, device=x.device), b.columns["index"].long() % self.chunk] = x
            return blk

        return make_batch_lambda(f, val)

    def make_output(self, keys, values):
        return RecordBatch({"chunk": keys, "block": values}, len(values))


class CommentInferenceJoin(JoinComp):
    def get_selection(self, r, c):
        return make_lambda_from_member(r, "index") == make_lambda_from_member(c, "index")

    def get_projection(self, r, c):
        def proj(rb, cb):
            cols = dict(cb.columns)
            cols["label"] = rb.columns["label"]
            return RecordBatch(cols, cb.n, RedditComment)

        return make_batch_lambda(r, c, proj)


class LabelSelection(SelectionComp):
    """RedditLabelSelection<p>_<t>: positive -> label < threshold, else label >= threshold."""

    def __init__(self, threshold: int, positive: bool = True):
        super().__init__()
        self.threshold, self.positive = threshold, positive

    def get_selection(self, c):
        lab = make_lambda_from_member(c, "label")
        return (lab < self.threshold) if self.positive else (lab >= self.threshold)

    def get_projection(self, c):
        return make_lambda_from_self(c)


class ThreeWayJoin(JoinComp):
    def __init__(self):
        super().__init__(3)

    def get_selection(self, c, a, s):
        return (make_lambda_from_member(c, "author") == make_lambda_from_member(a, "author")) & \
            (make_lambda_from_member(c, "subreddit_id") == make_lambda_from_member(s, "name"))

    def get_projection(self, c, a, s):
        def proj(cb, ab, sb):
            extra = torch.stack([ab.columns["comment_karma"].double(), ab.columns["link_karma"].double(),
                                 sb.columns["subscribers"].double()], 1)
            feats = torch.cat([comment_features(cb), torch.sign(extra) * torch.log1p(extra.abs())], 1)
            return RecordBatch({"index": cb.columns["index"], "author": cb.columns["author"],
                                "subreddit": cb.columns["subreddit_id"], "features": feats}, cb.n, FullFeatures)

        return make_batch_lambda(c, a, s, proj)


class CommentPartition(PartitionComp):
    """CommentPartition / AuthorCommentsPartition: repartition comments by index or author."""

    def __init__(self, db: str, set_name: str, by: str = "index"):
        super().__init__(db, set_name)
        self.by = by

    def get_key_projection(self, c):
        return make_lambda_from_member(c, self.by)


# -------------------------------------------------------------------------------- data + driver
def generate(n_comments: int = 500, n_authors: int = 40, n_subs: int = 8, seed: int = 0) -> Dict[str, RecordBatch]:
    g = torch.Generator().manual_seed(seed)
    authors = [f"user{i}" for i in range(n_authors)]
    subs = [f"t5_{i:04x}" for i in range(n_subs)]
    ai = torch.randint(0, n_authors, (n_comments,), generator=g)
    si = torch.randint(0, n_subs, (n_comments,), generator=g)
    created = torch.randint(1_300_000_000, 1_600_000_000, (n_comments,), generator=g)
    comments = RecordBatch({
        "index": torch.arange(n_comments), "label": torch.zeros(n_comments, dtype=torch.int64),
        "author": [authors[i] for i in ai.tolist()], "subreddit_id": [subs[i] for i in si.tolist()],
        "author_created_utc": created - torch.randint(0, 300_000_000, (n_comments,), generator=g),
        "created_utc": created, "retrieved_on": created + torch.randint(0, 10_000_000, (n_comments,), generator=g),
        "score": torch.randint(-50, 500, (n_comments,), generator=g),
        "controversiality": torch.randint(0, 2, (n_comments,), generator=g),
        "gilded": torch.randint(0, 3, (n_comments,), generator=g),
        "archived": torch.randint(0, 2, (n_comments,), generator=g),
        "body": [f"comment {i}" for i in range(n_comments)]}, n_comments, RedditComment)
    authors_b = RecordBatch({"author": authors, "comment_karma": torch.randint(0, 100000, (n_authors,), generator=g),
                             "link_karma": torch.randint(0, 100000, (n_authors,), generator=g),
                             "created_utc": torch.randint(1_100_000_000, 1_300_000_000, (n_authors,), generator=g)},
                            n_authors, RedditAuthor)
    subs_b = RecordBatch({"name": subs, "subscribers": torch.randint(10, 10_000_000, (n_subs,), generator=g),
                          "created_utc": torch.randint(1_100_000_000, 1_300_000_000, (n_subs,), generator=g)},
                         n_subs, RedditSub)
    return {"comments": comments, "authors": authors_b, "subs": subs_b}


def load(client, db: str, data: Dict[str, RecordBatch]):
    client.create_database(db)
    for name, typ in (("comments", RedditComment), ("authors", RedditAuthor), ("subs", RedditSub)):
        client.create_set(db, name, typ)
        client.send_data(db, name, data[name])


def _run(client, db, out, comp, job):
    if client.storage.has_set(db, out):
        client.remove_set(db, out)
    client.create_set(db, out, None)
    client.execute_computations(WriteSet(db, out).set_input(comp), job_name=job)
    got = [b for b in client.get_set_batches(db, out, gather=True) if b.n]
    if not got:
        return None
    b = RecordBatch.concat(got)
    if len(b.columns) == 1 and isinstance(next(iter(b.columns.values())), RecordBatch):
        b = next(iter(b.columns.values()))
    return b


def features_matrix(client, db: str, n: int, chunk: int = 64) -> torch.Tensor:
    """CommentsToFeatures -> CommentChunksToBlocks -> CommentBlockToMatrix: the [n, F] feature matrix."""
    feats = CommentsToFeatures().set_input(ScanSet(db, "comments", RedditComment))
    blocks = _run(client, db, "comment_blocks", CommentChunksToBlocks(chunk).set_input(feats), "reddit_features")
    X = torch.zeros(((n + chunk - 1) // chunk) * chunk, NUM_FEATURES, dtype=torch.float64)
    for k, blk in zip(blocks.columns["chunk"].tolist(), blocks.columns["block"].cpu()):
        X[k * chunk:(k + 1) * chunk] = blk
    return X[:n]


def infer_labels(client, db: str, n: int, hidden: int = 32, labels: int = 4, block: int = 16, seed: int = 0):
    """Feature matrix -> FF inference (random-init weights, as the reference's pipeline test) ->
    InferenceResult set -> CommentInferenceJoin -> labelled comments set ``labelled``."""
    X = features_matrix(client, db, n)
    mdb = f"{db}_ff"
    ff.setup(client, mdb)
    B.load_tensor(client, mdb, "inputs", X.float(), block, block, dtype=torch.float32)
    g = torch.Generator().manual_seed(seed)
    w1 = torch.randn(hidden, NUM_FEATURES, generator=g) * (3.0 / NUM_FEATURES) ** 0.5
    wo = torch.randn(labels, hidden, generator=g) * (3.0 / hidden) ** 0.5
    b1, bo = torch.randn(hidden, 1, generator=g) * 0.1, torch.randn(labels, 1, generator=g) * 0.1
    for nm, t in (("w1", w1), ("wo", wo), ("b1", b1), ("bo", bo)):
        B.load_tensor(client, mdb, nm, t, block, block if t.shape[1] > 1 else 1, dtype=torch.float32)
    ff.inference_unit(client, mdb, "w1", "wo", "inputs", "b1", "bo", "output")
    probs = B.to_tensor(client, mdb, "output").float()[:n, :labels]
    lab = probs.argmax(1)
    ref = ff.reference_inference(X.float(), w1, b1, wo, bo).argmax(1)
    if client.storage.has_set(db, "inference"):
        client.remove_set(db, "inference")
    client.create_set(db, "inference", InferenceResult)
    client.send_data(db, "inference", RecordBatch({"index": torch.arange(n), "label": lab.long()}, n, InferenceResult))
    j = CommentInferenceJoin()
    j.set_input(0, ScanSet(db, "inference", InferenceResult))
    j.set_input(1, ScanSet(db, "comments", RedditComment))
    out = _run(client, db, "labelled", j, "reddit_label_join")
    return out, lab, ref


def infer_results(client, db: str, n: int, hidden: int = 32, labels: int = 4, block: int = 16, seed: int = 0,
                  enable_partition: bool = False):
    """RedditFeatureExtractor.cc's inference stage: FF inference over the comment feature blocks, then
    FFMatrixMultiSel flattens the output blocks into one ff.InferenceResult per comment (row index + its first
    two scores), written by InferenceResultPartition (partitioned by index) when ``enable_partition``, else by a
    plain writer. Returns (results batch sorted by index, the fp32 reference scores [n, 2])."""
    X = features_matrix(client, db, n)
    mdb = f"{db}_ffr"
    ff.setup(client, mdb)
    B.load_tensor(client, mdb, "inputs", X.float(), block, block, dtype=torch.float32)
    g = torch.Generator().manual_seed(seed)
    w1 = torch.randn(hidden, NUM_FEATURES, generator=g) * (3.0 / NUM_FEATURES) ** 0.5
    wo = torch.randn(labels, hidden, generator=g) * (3.0 / hidden) ** 0.5
    b1, bo = torch.randn(hidden, 1, generator=g) * 0.1, torch.randn(labels, 1, generator=g) * 0.1
    for nm, t in (("w1", w1), ("wo", wo), ("b1", b1), ("bo", bo)):
        B.load_tensor(client, mdb, nm, t, block, block if t.shape[1] > 1 else 1, dtype=torch.float32)
    ff.inference_unit(client, mdb, "w1", "wo", "inputs", "b1", "bo", "output")
    if client.storage.has_set(mdb, "results"):
        client.remove_set(mdb, "results")
    client.create_set(mdb, "results", ff.InferenceResult)
    sel = ff.FFMatrixMultiSel().set_input(ff.FFMatrixBlockScanner(mdb, "output"))
    writer = ff.InferenceResultPartition(mdb, "results") if enable_partition else \
        WriteSet(mdb, "results", ff.InferenceResult)
    client.execute_computations(writer.set_input(sel), job_name="reddit_inference_results")
    got = [b for b in client.get_set_batches(mdb, "results", gather=True) if b.n]
    res = RecordBatch.concat(got)
    res = res.take(torch.argsort(res.columns["index"]))
    ref = ff.reference_inference(X.float(), w1, b1, wo, bo)[:, :2]
    return res, ref


def label_split(client, db: str, threshold: int) -> List[int]:
    pos = _run(client, db, "positives", LabelSelection(threshold, True).set_input(ScanSet(db, "labelled")),
               "reddit_label_pos")
    neg = _run(client, db, "negatives", LabelSelection(threshold, False).set_input(ScanSet(db, "labelled")),
               "reddit_label_neg")
    return [0 if pos is None else pos.n, 0 if neg is None else neg.n]


def full_features(client, db: str) -> RecordBatch:
    j = ThreeWayJoin()
    j.set_input(0, ScanSet(db, "comments", RedditComment))
    j.set_input(1, ScanSet(db, "authors", RedditAuthor))
    j.set_input(2, ScanSet(db, "subs", RedditSub))
    return _run(client, db, "full_features", j, "reddit_three_way_join")
