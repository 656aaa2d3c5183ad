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


class SoftmaxXentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, smoothing: float):
        B, NC = logits.shape
        lg = logits.float().contiguous()
        loss_rows = torch.empty(B, dtype=torch.float32, device=lg.device)
        dlog = torch.empty_like(lg)
        correct = torch.empty(B, dtype=torch.int32, device=lg.device)
        _native.kernels().softmax_xent(lg.data_ptr(), labels.contiguous().data_ptr(), loss_rows.data_ptr(),
                                       dlog.data_ptr(), correct.data_ptr(), B, NC, 1.0 / B, float(smoothing),
                                       _native.stream(lg))
        ctx.save_for_backward(dlog)
        ctx.in_dtype = logits.dtype
        ctx.mark_non_differentiable(correct)
        return loss_rows.mean(), correct

    @staticmethod
    def backward(ctx, dloss, _dc):
        (dlog,) = ctx.saved_tensors
        return (dlog * dloss).to(ctx.in_dtype), None, None


def softmax_xent(logits: torch.Tensor, labels: torch.Tensor, smoothing: float = 0.0, with_correct: bool = False):
    """Mean cross-entropy of ``logits`` [B, NC] against int64 ``labels`` [B].

    Dense predictions (per-voxel segmentation, ``logits`` [N, ..., NC] with
    ``labels`` [N, ...]) are flattened to one row per voxel.
    """
    if logits.dim() > 2:
        logits = logits.reshape(-1, logits.shape[-1])
        labels = labels.reshape(-1)
    if _native.use_native(logits):
        loss, correct = SoftmaxXentFn.apply(logits, labels.long(), smoothing)
        return (loss, correct) if with_correct else loss
    loss = ref.softmax_xent(logits, labels.long(), smoothing)
    if with_correct:
        return loss, (logits.argmax(-1) == labels).int()
    return loss
