"""Why does Q12's final aggregation leave the fused device group-by (execution/kernels.group_reduce)? Wraps
group_reduce and _hash_aggregate, runs Q12 at SF 1 on the GPU and prints their inputs / statuses."""
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netsdb_amd.client import PDBClient  # noqa: E402
from netsdb_amd.execution import kernels as K  # noqa: E402
from netsdb_amd.models import tpch, tpch_gen  # noqa: E402

orig_gr, orig_ha = K.group_reduce, K._hash_aggregate


def gr(keys, values, op="sum"):
    r = orig_gr(keys, values, op)
    ks = keys if isinstance(keys, tuple) else (keys,)
    print("group_reduce", op, [type(k).__name__ for k in ks], type(values).__name__,
          getattr(values, "shape", None), getattr(values, "dtype", None), getattr(values, "device", None),
          getattr(values, "stride", lambda: None)(), "->", "None" if r is None else "ok", flush=True)
    return r


def ha(key64, vals, op, want_inv, want_first=True):
    out = torch.ops  # noqa: F841
    from netsdb_amd import _ext
    r = _ext.hip().hash_aggregate(key64.contiguous(), vals, op, want_inv, 0, want_first)
    print("  hash_aggregate status", r[5].tolist(), flush=True)
    return orig_ha(key64, vals, op, want_inv, want_first)


K.group_reduce, K._hash_aggregate = gr, ha
t = tpch_gen.generate_fast(1.0, seed=1)
c = PDBClient(root=tempfile.mkdtemp(), device=torch.device("cuda:0"))
tpch.load(c, "tpch", t, device=torch.device("cuda:0"))
print(tpch.QUERIES["q12"](c, "tpch"))
