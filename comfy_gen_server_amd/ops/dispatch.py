"""Backend selection for the op layer.

Policy (per op, overridable with ``CGS_OP_<NAME>=hip|torch|lib`` or ``set_backend_override``):
  * CPU tensors            -> ``torch`` (fp32 reference math).
  * ROCm tensors           -> ``hip`` when the kernel exists in libcgs_kernels.so.
                              ``lib`` means the vendor library through ATen (hipBLASLt GEMM /
                              MIOpen conv) — allowed only for plain GEMM/conv shapes without a
                              fused epilogue, and only when selected explicitly.
  * ROCm tensor + missing native library -> ``NativeMissingError`` (loud), unless
    ``CGS_ALLOW_TORCH_FALLBACK=1``.
"""
from __future__ import annotations

import collections
import os
import threading

import torch

from .. import _native


class NativeMissingError(RuntimeError):
    pass


_overrides: dict[str, str] = {}
_stats = collections.Counter()
_stats_lock = threading.Lock()

# Ops whose default device path is the vendor library until the hand-written kernel beats it.
# Filled in from measurements (profiles/): see ops/core.py docstrings.
_DEFAULT_DEVICE_BACKEND: dict[str, str] = {}


def set_backend_override(op: str, backend: str | None):
    if backend is None:
        _overrides.pop(op, None)
    else:
        _overrides[op] = backend


def set_default_device_backend(op: str, backend: str):
    _DEFAULT_DEVICE_BACKEND[op] = backend


def native_required() -> bool:
    return os.environ.get("CGS_ALLOW_TORCH_FALLBACK", "0") != "1"


_reference_depth = 0


class torch_reference:
    """``with torch_reference():`` every op takes its ``torch`` path (fp32 math, device tensors included):
    the numerics oracle of the production-scale golden tests (tests/test_golden_sdxl_gpu.py)."""

    def __enter__(self):
        global _reference_depth
        _reference_depth += 1
        return self

    def __exit__(self, *a):
        global _reference_depth
        _reference_depth -= 1


def backend_for(op: str, t: torch.Tensor, kernel: str | None = None) -> str:
    """Pick the backend for op ``op`` given its primary input ``t``."""
    if t.device.type != "cuda" or _reference_depth > 0:
        return "torch"
    b = _overrides.get(op) or os.environ.get(f"CGS_OP_{op.upper()}") or _DEFAULT_DEVICE_BACKEND.get(op, "hip")
    if b == "hip":
        kname = kernel or f"cgs_{op}"
        if not _native.has_kernel(kname):
            if native_required():
                raise NativeMissingError(
                    f"HIP kernel {kname} unavailable ({_native.kernels_error()}); build with "
                    f"`python build_native.py` or set CGS_ALLOW_TORCH_FALLBACK=1")
            return "torch"
    return b


class VendorFallbackError(RuntimeError):
    pass


_warned: set = set()


def vendor_fallback(op: str, detail: str):
    """A device call of ``op`` is about to leave the hand-written kernels for a vendor library /
    ATen (SDPA, MIOpen, hipBLASLt, ...). Loud by design: logs once per (op, reason) and counts
    ``(op, "lib")``; with ``CGS_STRICT_NATIVE=1`` it raises instead (the GPU test tier and the
    flagship smoke run also assert zero ``lib`` calls on their paths)."""
    import logging
    if os.environ.get("CGS_STRICT_NATIVE", "0") == "1":
        raise VendorFallbackError(f"{op}: {detail} has no HIP kernel path (CGS_STRICT_NATIVE=1)")
    key = (op, detail)
    if key not in _warned:
        _warned.add(key)
        logging.warning("vendor fallback: %s (%s) runs through the vendor library, not a HIP kernel", op, detail)
    count(op, "lib")


def count(op: str, backend: str):
    with _stats_lock:
        _stats[(op, backend)] += 1


def stats() -> dict:
    with _stats_lock:
        return dict(_stats)


def reset_stats():
    with _stats_lock:
        _stats.clear()
