"""The GEMM STUDY build (module ``netsdb_amd._hip_study``, sources in ``csrc/study``): the diagnostic and rejected
variants of the block GEMM behind profiles/r2_gemm1_study and profiles/r3_w4a — 8-phase ablations, ring buffers,
cache policies, K-tail stealing, adaptive split-K, the in-launch split-K fix-up, the 4-wave structures and the
kernel studies. The product never imports it (``netsdb_amd.ops`` runs ``_hip_kernels`` only, whose
launcher exports the production configs and takes every launch decision as a per-call argument); A/B scripts
and the study tests use this module.
"""
from __future__ import annotations

import importlib

import torch

from . import ops

_mod = None


def ext():
    """The study extension (raises if it was not built: ``NSDB_BUILD=study python setup.py build_ext --inplace``)."""
    global _mod
    if _mod is None:
        import torch  # noqa: F401  (the extension links against libtorch)

        try:
            _mod = importlib.import_module("netsdb_amd._hip_study")
        except ImportError as e:
            raise RuntimeError(f"netsdb_amd._hip_study is not built: {e}") from None
    return _mod


def gemm_nt(A, B, bias=None, bias_mode=ops.BIAS_NONE, act=ops.ACT_NONE, out_dtype=torch.bfloat16, alpha=1.0,
            dropout=0.0, seed=0, splits=0, out=None, accumulate=False, cfg=None):
    """ops.gemm_nt semantics under the study launcher with study config ``cfg`` (see study_bindings.cpp); None
    keeps the config set by ``ext().gemm_force_config`` (A/B scripts that force once and call many times)."""
    m = ext()
    if bias is not None and bias.dtype != torch.float32:
        bias = bias.float()
    A, B = ops.gemm_operands(A, B)
    if cfg is not None:
        m.gemm_force_config(int(cfg))
    try:
        return m.gemm_nt(A, B, bias, int(bias_mode if bias is not None else 0), ops.act_code(act),
                         out_dtype == torch.float32, float(alpha), float(dropout), int(seed), int(splits), out,
                         bool(accumulate))
    finally:
        if cfg is not None:
            m.gemm_force_config(-1)


__all__ = ["ext", "gemm_nt"]
