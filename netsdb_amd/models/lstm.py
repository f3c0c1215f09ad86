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
from ..computations import JoinComp
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


def lstm_inference(xs: torch.Tensor, hidden: int, seed: int = 0) -> dict:
    m = LSTMModel(xs.shape[-1], hidden, xs.device, seed)
    t0 = time.perf_counter()
    h, c = m.forward(xs)
    return {"h": h, "c": c, "seconds": time.perf_counter() - t0, "model": m}


__all__ = ["LSTMThreeWaySum", "LSTMTwoSum", "LSTMHiddenState", "LSTMModel", "lstm_inference"]
