"""Loader for the in-tree native extensions.

* ``_hip_kernels`` — CDNA4 HIP kernels. On a machine with a GPU the HIP path is mandatory:
  :func:`hip` raises instead of silently falling back to eager PyTorch.
* ``_native`` — host C++ runtime (page pool, page files, TCAP parser, hash partitioner).
"""
from __future__ import annotations

import importlib

_hip_mod = None
_hip_err: Exception | None = None
_native_mod = None
_native_err: Exception | None = None


def _try_import(name):
    try:
        return importlib.import_module(f"netsdb_amd.{name}"), None
    except Exception as e:  # pragma: no cover - depends on build state
        return None, e


def gpu_present() -> bool:
    """True when a GPU is visible. Uses device_count (does not initialise HIP on this image)."""
    try:
        import torch

        return torch.cuda.device_count() > 0
    except Exception:
        return False


def hip():
    """Return the HIP kernel module; raise loudly if it is missing."""
    global _hip_mod, _hip_err
    if _hip_mod is None and _hip_err is None:
        import torch  # noqa: F401  (the extension links against libtorch)

        _hip_mod, _hip_err = _try_import("_hip_kernels")
    if _hip_mod is None:
        raise RuntimeError(
            "netsdb_amd._hip_kernels is not built (run `python setup.py build_ext --inplace` or "
            f"__graft_entry__.build()): {_hip_err}"
        )
    return _hip_mod


def hip_available() -> bool:
    try:
        hip()
        return True
    except RuntimeError:
        return False


def native():
    """Return the host C++ runtime module; raise if missing."""
    global _native_mod, _native_err
    if _native_mod is None and _native_err is None:
        _native_mod, _native_err = _try_import("_native")
    if _native_mod is None:
        raise RuntimeError(
            "netsdb_amd._native is not built (run `python setup.py build_ext --inplace`): " f"{_native_err}"
        )
    return _native_mod


def native_available() -> bool:
    try:
        native()
        return True
    except RuntimeError:
        return False

