"""Fused softmax + categorical cross-entropy.

Reference parity: the Keras head ``Dense(n, softmax)`` + ``categorical_crossentropy``
compiled in ``tensorflow_generator.py:232-235``.  The framework keeps logits and
fuses the softmax into the loss (numerically stable log-sum-exp); the GPU kernel
produces the mean loss, d(logits) and per-row top-1 hits in ONE pass, so
backward is a scale of a stored tensor.
"""
from __future__ import annotations

import torch

from .. import _native
from . import reference as ref


_UNIT: dict = {}


def unit_grad(t: torch.Tensor) -> torch.Tensor:
    """A cached device scalar 1.0 of ``t``'s dtype: ``loss.backward(unit_grad(loss))`` seeds the
    backward with a gradient the fused losses recognise (:func:`is_unit`) -- no ``ones_like`` fill
    launch, and no in-place scale of the stored d(logits)."""
    key = (str(t.device), t.dtype)
    u = _UNIT.get(key)
    if u is None:
        u = _UNIT[key] = torch.ones((), dtype=t.dtype, device=t.device)
    return u


def is_unit(d: torch.Tensor | None) -> bool:
    """True when ``d`` is the :func:`unit_grad` scalar itself (identity, not value: no sync)."""
    if d is None or d.dim() != 0:
        return False
    u = _UNIT.get((str(d.device), d.dtype))
    return u is not None and u.data_ptr() == d.data_ptr()


def backward(loss: torch.Tensor) -> None:
    """``loss.backward()`` seeded with :func:`unit_grad` (scalar losses)."""
    loss.backward(unit_grad(loss) if loss.dim() == 0 and loss.is_floating_point() else None)


def _xent_rows(lg, labels, smoothing, want_correct):
    """One pass of the fused kernel: (per-block loss partials -- or, with one block, the mean
    loss itself --, d(logits) with 1/B folded in, per-row top-1 hits or None)."""
    B, NC = lg.shape
    K = _native.kernels()
    nblk = K.softmax_xent_blocks(B, NC)
    part = torch.empty(max(int(nblk), 1), dtype=torch.float32, device=lg.device)
    dlog = torch.empty_like(lg)                         # 1/B folded in, logits' dtype
    correct = torch.empty(B, dtype=torch.int32, device=lg.device) if want_correct else None
    K.softmax_xent_rows(lg.data_ptr(), int(lg.dtype == torch.bfloat16), labels.data_ptr(),
                        part.data_ptr(), dlog.data_ptr(), _native.ptr(correct), B, NC, 1.0 / B,
                        float(smoothing), _native.stream(lg))
    return part, dlog, correct


class SoftmaxXentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, smoothing: float, want_correct: bool = True):
        B, NC = logits.shape
        lg = logits.contiguous()
        if lg.dtype not in (torch.bfloat16, torch.float32):
            lg = lg.float()
        labels = labels.contiguous()
        part, dlog, correct = _xent_rows(lg, labels, smoothing, want_correct)
        # logits / labels are kept only for a second backward (retain_graph), which recomputes
        # d(logits): the first backward scales the stored one in place
        ctx.save_for_backward(dlog, lg, labels)
        ctx.in_dtype = logits.dtype
        ctx.smoothing = smoothing
        if correct is not None:
            ctx.mark_non_differentiable(correct)
        # one block (classifier batches): the kernel wrote the mean itself
        return (part.view(()) if part.numel() == 1 else part.sum() / B), correct

    @staticmethod
    def backward(ctx, dloss, _dc):
        dlog, lg, labels = ctx.saved_tensors
        if getattr(ctx, "scaled", False):
            # a second backward (retain_graph): the stored d(logits) already carries the first
            # call's dloss, so recompute it and scale out of place
            _, base, _ = _xent_rows(lg, labels, ctx.smoothing, False)
            return (base * dloss.to(base.dtype)).to(ctx.in_dtype), None, None, None
        ctx.scaled = True
        # scale the stored d(logits) in place by dloss -- nothing at all for the unit seed
        # (loss.backward(unit_grad(loss))), else a near-empty launch when dloss == 1 (a plain
        # loss.backward()): the device-side check needs no host sync
        if not is_unit(dloss):
            s = dloss.detach().float().reshape(1).contiguous()
            _native.kernels().scale_unless_one(dlog.data_ptr(), int(dlog.dtype == torch.bfloat16), s.data_ptr(),
                                               dlog.numel(), _native.stream(dlog))
        return dlog.to(ctx.in_dtype), None, None, None


def softmax_xent(logits: torch.Tensor, labels: torch.Tensor, smoothing: float = 0.0, with_correct: bool = False):
    """Mean cross-entropy of ``logits`` [B, NC] against int64 ``labels`` [B].

    Dense predictions (per-voxel segmentation, ``logits`` [N, ..., NC] with
    ``labels`` [N, ...]) are flattened to one row per voxel.
    """
    if logits.dim() > 2:
        logits = logits.reshape(-1, logits.shape[-1])
        labels = labels.reshape(-1)
    if _native.use_native(logits):
        loss, correct = SoftmaxXentFn.apply(logits, labels.long(), smoothing, with_correct)
        return (loss, correct) if with_correct else loss
    loss = ref.softmax_xent(logits, labels.long(), smoothing)
    if with_correct:
        return loss, (logits.argmax(-1) == labels).int()
    return loss
