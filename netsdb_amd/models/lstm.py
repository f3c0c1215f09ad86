"""LSTM inference (reference: src/LSTM — LSTMThreeWaySum (act(W·x + U·h + b) per gate),
LSTMTwoSum (c = f∘c_prev + i∘g), LSTMHiddenState (h = o∘tanh(c)); driver src/tests/source/LSTMTest.cc).

UDF classes are provided for the generic engine; the fast path runs one time step as ONE fused
GEMM over the concatenated [x_t | h_{t-1}] with the stacked gate weights [W | U] and bias in the
epilogue (all four gates at once), followed by the fused ``lstm_cell`` HIP kernel.
"""
from __future__ import annotations

import time

import torch

from .. import ops
from ..computations import CellUpdate, GateSum, HiddenOut, JoinComp
from ..lambdas import make_batch_lambda, make_lambda_from_method
from ..objects.record import RecordBatch
from .ff import mk_blocks


class LSTMThreeWaySum(JoinComp):
    """act(in1 + in2 + in3) for blocks with equal keys (sigmoid or tanh)."""

    def __init__(self, activation: str = "sigmoid"):
        super().__init__(3)
        self.activation = activation

    def get_selection(self, a, b, c):
        return (make_lambda_from_method(a, "getKey") == make_lambda_from_method(b, "getKey")) & \
               (make_lambda_from_method(a, "getKey") == make_lambda_from_method(c, "getKey"))

    def get_projection(self, a, b, c):
        def proj(x: RecordBatch, y: RecordBatch, z: RecordBatch):
            s = x.columns["data"].float() + y.columns["data"].float() + z.columns["data"].float()
            s = torch.sigmoid(s) if self.activation == "sigmoid" else torch.tanh(s)
            return mk_blocks(x.columns["block_row"], x.columns["block_col"], s, x.columns["total_rows"],
                             x.columns["total_cols"])

        return make_batch_lambda(a, b, c, proj, tag=f"threeway_{self.activation}")

    def tensor_pattern(self):
        return GateSum(act=self.activation)


class LSTMTwoSum(JoinComp):
    """c = f∘c_prev + i∘g (inputs: f, c_prev, i, g)."""

    def __init__(self):
        super().__init__(4)

    def get_selection(self, f, cp, i, g):
        k = make_lambda_from_method(f, "getKey")
        return (k == make_lambda_from_method(cp, "getKey")) & (k == make_lambda_from_method(i, "getKey")) & \
               (k == make_lambda_from_method(g, "getKey"))

    def get_projection(self, f, cp, i, g):
        def proj(F: RecordBatch, C: RecordBatch, I: RecordBatch, G: RecordBatch):
            d = F.columns["data"].float() * C.columns["data"].float() + I.columns["data"].float() * G.columns["data"].float()
            return mk_blocks(F.columns["block_row"], F.columns["block_col"], d, F.columns["total_rows"],
                             F.columns["total_cols"])

        return make_batch_lambda(f, cp, i, g, proj, tag="lstm_two_sum")

    def tensor_pattern(self):
        return CellUpdate()


class LSTMHiddenState(JoinComp):
    """h = o∘tanh(c)."""

    def get_selection(self, o, c):
        return make_lambda_from_method(o, "getKey") == make_lambda_from_method(c, "getKey")

    def get_projection(self, o, c):
        def proj(O: RecordBatch, C: RecordBatch):
            d = O.columns["data"].float() * torch.tanh(C.columns["data"].float())
            return mk_blocks(O.columns["block_row"], O.columns["block_col"], d, O.columns["total_rows"],
                             O.columns["total_cols"])

        return make_batch_lambda(o, c, proj, tag="lstm_hidden")

    def tensor_pattern(self):
        return HiddenOut()


class LSTMModel:
    """Stacked-gate LSTM weights: W [4H, D], U [4H, H], b [4H] (gate order i, f, g, o)."""

    def __init__(self, input_dim: int, hidden: int, device="cpu", seed: int = 0, dtype=torch.bfloat16):
        g = torch.Generator(device=device).manual_seed(seed)
        s = 1.0 / hidden ** 0.5
        self.D, self.H = input_dim, hidden
        self.W = (torch.rand(4 * hidden, input_dim, generator=g, device=device) * 2 - 1) * s
        self.U = (torch.rand(4 * hidden, hidden, generator=g, device=device) * 2 - 1) * s
        self.b = (torch.rand(4 * hidden, generator=g, device=device) * 2 - 1) * s
        # fused operand: one K-contiguous [4H, D+H (padded)] weight panel
        self.WU = ops.pad_k(torch.cat([self.W, self.U], 1)).to(dtype).contiguous()
        self.dtype = dtype

    def step(self, x: torch.Tensor, h: torch.Tensor, c: torch.Tensor):
        xh = ops.pad_k(torch.cat([x.to(self.dtype), h.to(self.dtype)], 1)).contiguous()
        gates = ops.gemm_nt(xh, self.WU, self.b.float(), ops.BIAS_COL, out_dtype=torch.float32)
        h2, c2 = ops.lstm_cell(gates, c.float().contiguous())
        return h2, c2

    def forward(self, xs: torch.Tensor):
        """xs [T, B, D] -> (h_T, c_T)."""
        T, B, _ = xs.shape
        h = torch.zeros(B, self.H, device=xs.device)
        c = torch.zeros(B, self.H, device=xs.device)
        for t in range(T):
            h, c = self.step(xs[t], h, c)
        return h, c

    def reference(self, xs: torch.Tensor):
        T, B, _ = xs.shape
        h = torch.zeros(B, self.H, dtype=torch.float64)
        c = torch.zeros(B, self.H, dtype=torch.float64)
        W, U, b = self.W.double().cpu(), self.U.double().cpu(), self.b.double().cpu()
        for t in range(T):
            gts = xs[t].double().cpu() @ W.t() + h @ U.t() + b
            i, f, g, o = gts.chunk(4, 1)
            c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
            h = torch.sigmoid(o) * torch.tanh(c)
        return h, c


# ------------------------------------------------------------------ the LSTMTest.cc job graph through the DB
GATES = {"f": "sigmoid", "i": "sigmoid", "o": "sigmoid", "c": "tanh"}     # c = the candidate (c_t_temp)


def load_lstm_sets(client, db: str, D: int, B: int, L: int, block_x: int = 100, block_y: int = 100, seed: int = 0,
                   dtype=torch.float32):
    """LSTMTest.cc: w_{f,i,o,c} [L x D], u_* [L x L], b_* [L x B] (full bias matrices), x_t [D x B],
    h_t_1 and c_t_1 [L x B] — random (loadMatrix) dense FFMatrixBlock sets."""
    from . import blocks as Bk
    from .ff import setup

    setup(client, db)
    g = 0
    for k in GATES:
        Bk.load_matrix(client, db, f"w_{k}", L, D, block_x, block_y, seed=seed + g, scale=D ** -0.5, dtype=dtype)
        Bk.load_matrix(client, db, f"u_{k}", L, L, block_x, block_y, seed=seed + g + 1, scale=L ** -0.5, dtype=dtype)
        Bk.load_matrix(client, db, f"b_{k}", L, B, block_x, block_y, seed=seed + g + 2, scale=0.1, dtype=dtype)
        g += 3
    Bk.load_matrix(client, db, "x_t", D, B, block_x, block_y, seed=seed + 20, dtype=dtype)
    Bk.load_matrix(client, db, "h_t_1", L, B, block_x, block_y, seed=seed + 21, scale=0.5, dtype=dtype)
    Bk.load_matrix(client, db, "c_t_1", L, B, block_x, block_y, seed=seed + 22, scale=0.5, dtype=dtype)


def _gate_comp(db: str, k: str):
    from .ff import FFAggMatrix, FFInputLayerJoin, FFMatrixBlockScanner

    jw = FFInputLayerJoin()
    jw.set_input(0, FFMatrixBlockScanner(db, f"w_{k}"))
    jw.set_input(1, FFMatrixBlockScanner(db, "x_t"))
    ju = FFInputLayerJoin()
    ju.set_input(0, FFMatrixBlockScanner(db, f"u_{k}"))
    ju.set_input(1, FFMatrixBlockScanner(db, "h_t_1"))
    s = LSTMThreeWaySum(GATES[k])
    s.set_input(0, FFAggMatrix().set_input(jw))
    s.set_input(1, FFAggMatrix().set_input(ju))
    s.set_input(2, FFMatrixBlockScanner(db, f"b_{k}"))
    return s


def lstm_step_jobs(client, db: str) -> list:
    """The reference's job sequence (LSTMTest.cc:165-420): one job per gate (FFInputLayerJoin + FFAggMatrix
    for W.x and U.h, LSTMThreeWaySum with the bias set) writing f_t, i_t, o_t, c_t_temp; then LSTMTwoSum
    -> c_t and LSTMHiddenState -> h_t.  Each gate job lowers to ONE MFMA GEMM over [W | U] . [x ; h] with
    the bias matrix + activation in its epilogue."""
    from .ff import FFMatrixBlockScanner, FFMatrixWriter, create_output_set

    stats = []
    out_names = {"f": "f_t", "i": "i_t", "o": "o_t", "c": "c_t_temp"}
    for k, name in out_names.items():
        create_output_set(client, db, name)
        stats.append(client.execute_computations(FFMatrixWriter(db, name).set_input(_gate_comp(db, k)),
                                                 job_name=f"lstm-gate-{k}"))
    create_output_set(client, db, "c_t")
    two = LSTMTwoSum()
    for i, n in enumerate(("f_t", "c_t_1", "i_t", "c_t_temp")):
        two.set_input(i, FFMatrixBlockScanner(db, n))
    stats.append(client.execute_computations(FFMatrixWriter(db, "c_t").set_input(two), job_name="lstm-two-sum"))
    create_output_set(client, db, "h_t")
    hid = LSTMHiddenState()
    hid.set_input(0, FFMatrixBlockScanner(db, "o_t"))
    hid.set_input(1, FFMatrixBlockScanner(db, "c_t"))
    stats.append(client.execute_computations(FFMatrixWriter(db, "h_t").set_input(hid), job_name="lstm-hidden"))
    return stats


def lstm_step_graph(client, db: str):
    """The same time step as ONE computation graph (writers of c_t and h_t): lowers to one stacked gate
    GEMM ([W_i|U_i; W_f|U_f; W_c|U_c; W_o|U_o] . [x ; h], bias matrices in the epilogue) + ``lstm_cell``."""
    from .ff import FFMatrixBlockScanner, FFMatrixWriter, create_output_set

    gates = {k: _gate_comp(db, k) for k in GATES}
    two = LSTMTwoSum()
    two.set_input(0, gates["f"])
    two.set_input(1, FFMatrixBlockScanner(db, "c_t_1"))
    two.set_input(2, gates["i"])
    two.set_input(3, gates["c"])
    hid = LSTMHiddenState()
    hid.set_input(0, gates["o"])
    hid.set_input(1, two)
    create_output_set(client, db, "c_t")
    create_output_set(client, db, "h_t")
    return client.execute_computations(FFMatrixWriter(db, "c_t").set_input(two),
                                       FFMatrixWriter(db, "h_t").set_input(hid), job_name="lstm-step")


def lstm_db_reference(client, db: str):
    """fp64 reference of one step from the stored sets: (h_t, c_t) as [L x B]."""
    from .blocks import to_tensor

    g = lambda n: to_tensor(client, db, n).double().cpu()  # noqa: E731
    x, h, c = g("x_t"), g("h_t_1"), g("c_t_1")
    pre = {k: g(f"w_{k}") @ x + g(f"u_{k}") @ h + g(f"b_{k}") for k in GATES}
    f, i, o = (torch.sigmoid(pre[k]) for k in ("f", "i", "o"))
    cand = torch.tanh(pre["c"])
    c2 = f * c + i * cand
    return o * torch.tanh(c2), c2


def lstm_inference(xs: torch.Tensor, hidden: int, seed: int = 0) -> dict:
    m = LSTMModel(xs.shape[-1], hidden, xs.device, seed)
    t0 = time.perf_counter()
    h, c = m.forward(xs)
    return {"h": h, "c": c, "seconds": time.perf_counter() - t0, "model": m}


__all__ = ["LSTMThreeWaySum", "LSTMTwoSum", "LSTMHiddenState", "LSTMModel", "lstm_inference", "load_lstm_sets",
           "lstm_step_jobs", "lstm_step_graph", "lstm_db_reference"]
