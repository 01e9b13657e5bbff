"""Loader for the in-tree CDNA4 kernel library ``symmetry_amd/_C.so``.

The library registers ``torch.ops.symmetry_amd.*``.  On a GPU tensor every op
in :mod:`symmetry_amd.ops` dispatches to it and raises if it is missing --
there is no silent eager fallback on the device.  CPU tensors use the fp32
torch references in :mod:`symmetry_amd.ops.reference` (tests, tiny models).
"""
from __future__ import annotations

import os
import threading

import torch

_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_C.so")
_lock = threading.Lock()
_loaded = False
_error: str | None = None


def load(build_if_missing: bool = False) -> bool:
    """Load ``_C.so`` once.  Returns True when the kernels are registered."""
    global _loaded, _error
    with _lock:
        if _loaded:
            return True
        if not os.path.exists(_LIB) and build_if_missing:
            from symmetry_amd import _build

            _build.build_kernels()
        if not os.path.exists(_LIB):
            _error = f"{_LIB} not built (run `python -m symmetry_amd._build`)"
            return False
        try:
            torch.ops.load_library(_LIB)
        except Exception as exc:  # pragma: no cover - depends on the box
            _error = f"failed to load {_LIB}: {exc}"
            return False
        _loaded = True
        return True


def available() -> bool:
    return load()


def ops():
    """Return ``torch.ops.symmetry_amd`` or raise loudly."""
    if not load():
        raise RuntimeError(f"symmetry_amd native kernels unavailable: {_error}")
    return torch.ops.symmetry_amd


def library_path() -> str:
    return _LIB
