"""Loading of the in-tree native modules.

``_hipops`` (HIP kernels for gfx950) is REQUIRED for any op on a GPU tensor:
if it is missing or fails to load on a machine with a GPU, ops raise instead
of silently falling back to PyTorch. ``_pscore`` is the host C++ runtime.
"""
from __future__ import annotations

import importlib
import os

_hip = None
_hip_err: Exception | None = None
_core = None


def hipops():
    """The HIP kernel module; raises loudly if it cannot be loaded."""
    global _hip, _hip_err
    if _hip is None and _hip_err is None:
        try:
            import torch  # noqa: F401  (libtorch must be loaded first)

            _hip = importlib.import_module("parameter_server_amd._hipops")
        except Exception as e:  # pragma: no cover - exercised on broken builds only
            _hip_err = e
    if _hip is None:
        raise RuntimeError(
            "parameter_server_amd: HIP extension _hipops is not available "
            f"({_hip_err!r}); build it with `python -m parameter_server_amd._build`")
    return _hip


def core():
    """The host C++ runtime module (_pscore)."""
    global _core
    if _core is None:
        _core = importlib.import_module("parameter_server_amd._pscore")
    return _core


def hip_available() -> bool:
    try:
        hipops()
        return True
    except RuntimeError:
        return False


def is_gpu(t) -> bool:
    return bool(getattr(t, "is_cuda", False))


def ptr(t) -> int:
    """Raw address of a contiguous CPU tensor / ndarray (0 for None)."""
    if t is None:
        return 0
    if hasattr(t, "data_ptr"):
        assert t.is_contiguous(), "buffer must be contiguous"
        return t.data_ptr()
    return t.ctypes.data


def strict_native() -> bool:
    """On a GPU box the HIP path must be used; PSAMD_ALLOW_TORCH_FALLBACK=1 opts out."""
    return os.environ.get("PSAMD_ALLOW_TORCH_FALLBACK", "0") != "1"
