"""Loader for the in-tree HIP extension ``fraud_detection_amd._fdx_native``.

torch must be imported before the extension: torch bundles ``libamdhip64.so.7`` with the same
SONAME as /opt/rocm, and loading torch first makes the extension bind to that already-loaded
HIP runtime (one HIP context, torch's streams are valid handles for our launches).

Policy: tensors on a ROCm device MUST run through the native kernels.  If the extension is
missing or was built for another arch, device calls raise ``NativeUnavailableError`` instead of
silently falling back to eager PyTorch.  CPU tensors use the oracles in ``ops/reference.py``.
"""
from __future__ import annotations

import importlib
import os
import threading

import torch

_lock = threading.Lock()
_mod = None
_err: Exception | None = None


class NativeUnavailableError(RuntimeError):
    pass


def _load():
    global _mod, _err
    with _lock:
        if _mod is not None or _err is not None:
            return
        try:
            _mod = importlib.import_module("fraud_detection_amd._fdx_native")
        except Exception as e:  # pragma: no cover - exercised when the .so is absent
            _err = e


def native():
    """Return the extension module or raise NativeUnavailableError."""
    _load()
    if _mod is None:
        raise NativeUnavailableError(
            "fraud_detection_amd._fdx_native is not built/importable "
            f"({_err!r}); run `python -m fraud_detection_amd.build_native`"
        )
    return _mod


def available() -> bool:
    _load()
    return _mod is not None


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_of(t: torch.Tensor) -> int:
    """hipStream_t (as int) of torch's current stream on t's device.  The raw-handle query skips
    building a torch Stream object (a few us of host time per launch on the fit's critical path,
    profiles/r2_s6/host_profile_*.txt)."""
    idx = t.device.index
    if _raw_stream is not None and idx is not None:
        return int(_raw_stream(idx))
    return torch.cuda.current_stream(t.device).cuda_stream


def ptr(t: torch.Tensor | None) -> int:
    return 0 if t is None else int(t.data_ptr())


def on_gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


def require_gpu_native(t: torch.Tensor):
    """Return the native module for a device tensor (never falls back)."""
    if not t.is_cuda:
        raise ValueError("require_gpu_native called with a CPU tensor")
    m = native()
    return m


def check(cond: bool, msg: str) -> None:
    if not cond:
        raise ValueError(msg)


def force_cpu_reference() -> bool:
    """FDX_FORCE_REFERENCE=1 routes even device tensors through the CPU oracle (debug only)."""
    return os.environ.get("FDX_FORCE_REFERENCE", "0") == "1"
