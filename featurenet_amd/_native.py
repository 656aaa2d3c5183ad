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


def copy_in(dst0: torch.Tensor, src0: torch.Tensor, dst1: torch.Tensor | None = None,
            src1: torch.Tensor | None = None) -> None:
    """``dst0.copy_(src0)`` (and ``dst1.copy_(src1)``) as ONE native launch (``misc.hip``
    copy2_kernel) when both pairs are same-dtype, same-size, contiguous, 16-B aligned device
    tensors -- the training step's batch copy-in; otherwise torch's copies."""
    pairs = [(dst0, src0)] + ([(dst1, src1)] if dst1 is not None else [])
    ok = all(d.is_cuda and s.is_cuda and d.dtype == s.dtype and d.numel() == s.numel() and d.is_contiguous()
             and s.is_contiguous() and d.device == s.device and (d.data_ptr() | s.data_ptr()) % 16 == 0
             for d, s in pairs) and kernels_available()
    if not ok:
        for d, s in pairs:
            d.copy_(s)
        return
    nb = [d.numel() * d.element_size() for d, _ in pairs]
    d1, s1, n1 = (pairs[1][0].data_ptr(), pairs[1][1].data_ptr(), nb[1]) if len(pairs) > 1 else (0, 0, 0)
    kernels().copy2(dst0.data_ptr(), src0.data_ptr(), nb[0], d1, s1, n1, stream(dst0))
