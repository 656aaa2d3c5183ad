"""Dense layer: ``y = act(x @ W^T + b)``.

Reference parity: Keras ``Dense`` (``model/input.py:174-190``) and the
classifier head ``Dense(n_classes, softmax)`` (``model/keras_model.py:124``).

GPU: the matmul itself is a plain library GEMM (hipBLASLt through
``torch.matmul`` on bf16 operands, fp32 accumulate -- the brief reserves
hand-written MFMA kernels for the fused hot ops and lets plain GEMMs go to
the vendor library); bias + activation run in the native ``bias_act`` kernel
and the activation backward in ``act_bwd``.  The weight gradient is produced
in fp32 for the fp32 master weights.
"""
from __future__ import annotations

import torch

from .. import _native
from . import reference as ref
from .spec import act_code


class LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act: int, out_fp32: bool):
        wb = w.detach().to(torch.bfloat16)
        xb = x.to(torch.bfloat16)
        y = torch.matmul(xb, wb.t())
        if b is not None or act:
            y2 = torch.empty_like(y)
            _native.kernels().bias_act(y.data_ptr(), _native.ptr(b.detach().float().contiguous() if b is not None else None),
                                       y2.data_ptr(), y.numel(), y.shape[-1], act, _native.stream(y))
            y = y2
        ctx.save_for_backward(xb, wb, y if act else None)
        ctx.act, ctx.has_b = act, b is not None
        return y.float() if out_fp32 else y

    @staticmethod
    def backward(ctx, dy):
        xb, wb, y = ctx.saved_tensors
        dy = dy.to(torch.bfloat16).contiguous()
        if ctx.act:
            g = torch.empty_like(dy)
            _native.kernels().act_bwd(dy.data_ptr(), y.data_ptr(), g.data_ptr(), dy.numel(), ctx.act,
                                      _native.stream(dy))
            dy = g
        dx = torch.matmul(dy, wb) if ctx.needs_input_grad[0] else None
        dy2 = dy.reshape(-1, dy.shape[-1])
        x2 = xb.reshape(-1, xb.shape[-1])
        dw = torch.matmul(dy2.t(), x2).float() if ctx.needs_input_grad[1] else None
        db = dy2.float().sum(0) if (ctx.has_b and ctx.needs_input_grad[2]) else None
        return dx, dw, db, None, None


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None, act=None, out_fp32: bool = False):
    if _native.use_native(x):
        if act == "softmax":
            y = LinearFn.apply(x, w, b, 0, True)
            return torch.softmax(y, dim=-1)
        return LinearFn.apply(x, w, b, act_code(act), out_fp32)
    y = torch.nn.functional.linear(x, w.to(x.dtype), None if b is None else b.to(x.dtype))
    return ref.activation(y, act)
