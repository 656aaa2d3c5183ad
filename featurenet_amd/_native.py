"""Loader for the in-tree native libraries.

``kernels()`` returns the gfx950 HIP kernel module (``_C``).  On a machine
with a visible GPU a missing or broken kernel library is a hard error: the
framework never silently falls back to PyTorch kernels for GPU tensors (set
``FEATURENET_ALLOW_TORCH_FALLBACK=1`` to opt into the slow reference path for
debugging).  CPU tensors always use the PyTorch reference implementations in
:mod:`featurenet_amd.ops.reference` -- that is the framework's "CPU reference
path" (BASELINE.json config 1).
"""
from __future__ import annotations

import importlib
import os

import torch

_K = None
_RT = None
_K_ERR: Exception | None = None


def kernels():
    """Return the HIP kernel module, importing (never building) it."""
    global _K, _K_ERR
    if _K is not None:
        return _K
    try:
        _K = importlib.import_module("featurenet_amd._C")
    except Exception as e:  # pragma: no cover - exercised on GPU boxes only
        _K_ERR = e
        raise RuntimeError(
            "featurenet_amd HIP kernels are not built (python -m featurenet_amd._build): " + repr(e)
        ) from e
    return _K


def kernels_available() -> bool:
    try:
        kernels()
        return True
    except RuntimeError:
        return False


def runtime():
    """Return the host-side native runtime module (``_rt``)."""
    global _RT
    if _RT is None:
        _RT = importlib.import_module("featurenet_amd._rt")
    return _RT


def runtime_available() -> bool:
    try:
        runtime()
        return True
    except Exception:
        return False


def use_native(t: torch.Tensor) -> bool:
    """True when ``t`` must go through the native HIP path."""
    if not t.is_cuda:
        return False
    if os.environ.get("FEATURENET_ALLOW_TORCH_FALLBACK") == "1" and not kernels_available():
        return False
    return True


def stream(t: torch.Tensor | None = None) -> int:
    dev = t.device if t is not None else None
    return torch.cuda.current_stream(dev).cuda_stream


def ptr(t: torch.Tensor | None) -> int:
    return 0 if t is None else t.data_ptr()
