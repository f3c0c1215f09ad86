"""linearAlgebraDSL programs (reference samples src/linearAlgebraDSL/DSLSamples/test*.pdml and the
TestLA01..17 operator tests) evaluated through the engine vs an fp64 torch evaluation of the AST."""
import os

import pytest
import torch

from netsdb_amd.client import PDBClient
from netsdb_amd.la import LAInstance, parse

REF = "/root/reference/src/linearAlgebraDSL/DSLSamples"


def ref_eval(program, files=None):
    env = {}

    def ev(e):
        k = e[0]
        if k == "id":
            return env[e[1]]
        if k == "num":
            return e[1]
        if k == "init":
            kind, a = e[1], e[2]
            if kind == "identity":
                return torch.eye(a[0] * a[1], dtype=torch.float64)
            r, c = a[0] * a[2], a[1] * a[3]
            if kind == "ones":
                return torch.ones(r, c, dtype=torch.float64)
            if kind == "zeros":
                return torch.zeros(r, c, dtype=torch.float64)
            return files[a[4]].double()
        if k == "bin":
            x, y = ev(e[2]), ev(e[3])
            return {"+": lambda: x + y, "-": lambda: x - y, "*": lambda: x * y, "%*%": lambda: x @ y,
                    "'*": lambda: x.t() @ y}[e[1]]()
        if k == "post":
            x = ev(e[2])
            return x.t() if e[1] == "^T" else torch.linalg.inv(x)
        if k == "func":
            x = ev(e[2])
            return {"max": lambda: x.max().reshape(1, 1), "min": lambda: x.min().reshape(1, 1),
                    "rowMax": lambda: x.amax(1, keepdim=True), "rowMin": lambda: x.amin(1, keepdim=True),
                    "rowSum": lambda: x.sum(1, keepdim=True), "colMax": lambda: x.amax(0, keepdim=True),
                    "colMin": lambda: x.amin(0, keepdim=True), "colSum": lambda: x.sum(0, keepdim=True)}[e[1]]()
        if k == "dup":
            x = ev(e[2])
            n = e[3] * e[4]
            return x[:1].expand(n, x.shape[1]) if e[1] == "duplicateRow" else x[:, :1].expand(x.shape[0], n)
        raise ValueError(e)

    for name, expr in parse(program):
        env[name] = ev(expr)
    return env


def _samples():
    if not os.path.isdir(REF):
        return []
    out = []
    for f in sorted(os.listdir(REF)):
        if f.startswith("test") and f.endswith(".pdml"):
            txt = open(os.path.join(REF, f)).read()
            if "load" not in txt:
                out.append((f, txt))
    return out


@pytest.mark.parametrize("name,program", _samples() or [("inline", "A = ones(20,20,2,2)\nB = identity(20,2)\nC = A + B")])
def test_reference_samples(tmp_path, name, program):
    c = PDBClient(root=str(tmp_path))
    la = LAInstance(c, dtype=torch.float32)
    la.run(program)
    ref = ref_eval(program)
    for var, exp in ref.items():
        got = la.get(var).double().cpu()
        torch.testing.assert_close(got, exp, atol=1e-3, rtol=1e-3, msg=f"{name}:{var}")


def test_regression_program(tmp_path):
    """The L2 / nearest-neighbour style programs of DSLSamples with load() from block files."""
    torch.manual_seed(0)
    X = torch.rand(40, 8)
    y = torch.rand(40, 1)
    t = torch.rand(1, 8)
    Mm = torch.rand(8, 8) + torch.eye(8) * 3

    def write(path, mat, br, bc):
        with open(path, "w") as f:
            for i in range(mat.shape[0] // br):
                for j in range(mat.shape[1] // bc):
                    blk = mat[i * br:(i + 1) * br, j * bc:(j + 1) * bc]
                    f.write(f"{i} {j} " + " ".join(f"{v:.7f}" for v in blk.flatten().tolist()) + "\n")

    px, py, pt, pm = (str(tmp_path / n) for n in ("X.data", "y.data", "t.data", "M.data"))
    write(px, X, 10, 8)
    write(py, y, 10, 1)
    write(pt, t, 1, 8)
    write(pm, Mm, 8, 8)
    prog = f'''X = load(10,8,4,1,"{px}")
y = load(10,1,4,1,"{py}")
t = load(1,8,1,1,"{pt}")
M = load(8,8,1,1,"{pm}")
beta = (X '* X)^-1 %*% (X '* y)
D = X - duplicateRow(t,10,4)
i = min(rowSum(D %*% M * D))
G = X '* X
'''
    c = PDBClient(root=str(tmp_path))
    la = LAInstance(c, dtype=torch.float32)
    la.run(prog)
    ref = ref_eval(prog, {px: X, py: y, pt: t, pm: Mm})
    for var in ("beta", "D", "i", "G"):
        torch.testing.assert_close(la.get(var).double().cpu(), ref[var], atol=5e-3, rtol=5e-3, msg=var)
