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

import os

import torch

from .. import _native
from . import reference as ref
from .spec import act_code

_SPLITK = os.environ.get("FN_FC_SPLITK", "1") != "0"


def _skinny_matmul(xb: torch.Tensor, wb: torch.Tensor) -> torch.Tensor:
    """x [M, K] @ w^T for a small M*N and a huge K (FeatureNet-3D FC1: 128 x 64000 x 128).

    hipBLASLt tiles this with ~56 workgroups on a 256-CU part; a 16-way split of K as a
    batched GEMM with fp32 partials fills the chip (73 -> ~40 us, ``bench/fc_gemm.py``)."""
    M, K = xb.shape
    N = wb.shape[0]
    s = 16
    xs = xb.view(M, s, K // s).transpose(0, 1)
    ws = wb.view(N, s, K // s).permute(1, 2, 0)
    try:
        part = torch.bmm(xs, ws, out_dtype=torch.float32)
    except (TypeError, RuntimeError):
        part = torch.bmm(xs, ws).float()
    return part.sum(0).to(torch.bfloat16)


def _wgrad(dy2: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
    """fp32 dW = dy^T x straight out of the GEMM (no bf16 round trip, no cast pass)."""
    try:
        return torch.mm(dy2.t(), x2, out_dtype=torch.float32)
    except (TypeError, RuntimeError):
        return torch.matmul(dy2.t(), x2).float()


class LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act: int, out_fp32: bool):
        wb = w.detach().to(torch.bfloat16)
        xb = x.to(torch.bfloat16)
        if _SPLITK and xb.dim() == 2 and xb.shape[0] * wb.shape[0] <= 256 * 256 and xb.shape[1] >= 16384 \
                and xb.shape[1] % 16 == 0:
            y = _skinny_matmul(xb.contiguous(), wb)
        else:
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
        dw = _wgrad(dy2, x2) if ctx.needs_input_grad[1] else None
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
