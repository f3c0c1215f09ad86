"""Reddit in-database inference pipeline (reference src/reddit): features, chunking to blocks, FF
inference, label join, label selections, three-way join."""
import datetime

import torch

from netsdb_amd.client import PDBClient
from netsdb_amd.models import reddit as R


def test_time_features_match_gmtime():
    ts = torch.tensor([0, 951782400, 1600000000, 1330473600, 1456790399, 1709164800])
    for t, row in zip(ts.tolist(), R._time_features(ts)):
        d = datetime.datetime.fromtimestamp(t, datetime.timezone.utc)
        exp = [d.day / 31, d.second / 60, d.minute / 59, d.hour / 23, (d.month - 1) / 11, (d.year - 1900) / 2021,
               ((d.weekday() + 1) % 7) / 6, (d.timetuple().tm_yday - 1) / 365, 0]
        torch.testing.assert_close(row, torch.tensor(exp, dtype=torch.float64))


def test_reddit_pipeline(tmp_path):
    data = R.generate(260, seed=3)
    c = PDBClient(root=str(tmp_path), page_size=1 << 14)
    R.load(c, "rd", data)
    X = R.features_matrix(c, "rd", 260, chunk=32)
    torch.testing.assert_close(X, R.comment_features(data["comments"]))
    out, lab, ref = R.infer_labels(c, "rd", 260)
    assert out.n == 260 and bool((lab == ref).all())
    got = dict(zip(out.columns["index"].tolist(), out.columns["label"].tolist()))
    assert all(got[i] == int(lab[i]) for i in range(260))
    pos, neg = R.label_split(c, "rd", 2)
    assert pos == int((lab < 2).sum()) and pos + neg == 260
    full = R.full_features(c, "rd")
    assert full.n == 260 and full.columns["features"].shape == (260, R.NUM_FEATURES + 3)
