"""Activation, dropout and the branch-combination ops.

Reference parity: ``Activation`` (``model/operation.py:152-165``), ``Dropout``
(``:103-114``), ``Add`` / ``Concatenate`` / ``Multiply`` (``:214-248``),
``ZeroPadding2D`` (``:116-137``), ``K.zeros`` (``model/input.py:159-165``).

GPU: activation fwd/bwd and dropout (counter-hash mask regenerated in
backward, never stored) are native kernels; add/multiply/concat/pad are
memory-bound one-liners that torch already runs as single vectorised kernels
on the channels-last layout (concat = write-into-slice).
"""
from __future__ import annotations

import random

import torch

from .. import _native
from . import reference as ref
from .spec import ACT_CODES, act_code


class ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, act: int):
        xb = x.to(torch.bfloat16).contiguous()
        y = torch.empty_like(xb)
        _native.kernels().bias_act(xb.data_ptr(), 0, y.data_ptr(), xb.numel(), xb.shape[-1], act, _native.stream(xb))
        ctx.save_for_backward(y)
        ctx.act = act
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dy = dy.to(torch.bfloat16).contiguous()
        dx = torch.empty_like(dy)
        _native.kernels().act_bwd(dy.data_ptr(), y.data_ptr(), dx.data_ptr(), dy.numel(), ctx.act, _native.stream(dy))
        return dx, None


def activation(x: torch.Tensor, act) -> torch.Tensor:
    if act in (None, "none", "linear"):
        return x
    if _native.use_native(x) and act in ACT_CODES:
        return ActFn.apply(x, act_code(act))
    return ref.activation(x, act)


class DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p: float, seed: int, offset: int):
        xb = x.to(torch.bfloat16).contiguous()
        y = torch.empty_like(xb)
        _native.kernels().dropout(xb.data_ptr(), y.data_ptr(), xb.numel(), float(p), seed, offset, _native.stream(xb))
        ctx.p, ctx.seed, ctx.offset = p, seed, offset
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.to(torch.bfloat16).contiguous()
        dx = torch.empty_like(dy)
        # same (seed, offset, index) -> same mask; scale by 1/(1-p) again
        _native.kernels().dropout(dy.data_ptr(), dx.data_ptr(), dy.numel(), float(ctx.p), ctx.seed, ctx.offset,
                                  _native.stream(dy))
        return dx, None, None, None


_DROP_OFFSET = [0]


def dropout(x: torch.Tensor, p: float, training: bool, generator: random.Random | None = None) -> torch.Tensor:
    if not training or p <= 0.0:
        return x
    if p >= 1.0:
        return torch.zeros_like(x)
    if _native.use_native(x):
        rng = generator or random
        seed = rng.getrandbits(32)
        _DROP_OFFSET[0] = (_DROP_OFFSET[0] + 1) & 0xFFFFFFFF
        return DropoutFn.apply(x, p, seed, _DROP_OFFSET[0])
    return torch.nn.functional.dropout(x, p, True)


def add(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return a + b


def multiply(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return a * b


def concat(tensors, axis: int) -> torch.Tensor:
    return torch.cat(tensors, dim=axis)


def zero_pad(x5: torch.Tensor, pads) -> torch.Tensor:
    """Zero-pad spatial dims of a 5-D channels-last tensor; pads = (d, h, w) per side."""
    pd, ph, pw = pads
    return torch.nn.functional.pad(x5, (0, 0, pw, pw, ph, ph, pd, pd))


class Upsample2xFn(torch.autograd.Function):
    """Nearest x2 upsampling of a channels-last grid (``upsample2x`` kernels on GPU)."""

    @staticmethod
    def forward(ctx, x5):
        N, D, H, W, C = x5.shape
        xb = x5.to(torch.bfloat16).contiguous()
        y = torch.empty(N, 2 * D, 2 * H, 2 * W, C, dtype=torch.bfloat16, device=x5.device)
        _native.kernels().upsample2x(xb.data_ptr(), y.data_ptr(), N, D, H, W, C, 0, _native.stream(xb))
        ctx.shape = (N, D, H, W, C)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, D, H, W, C = ctx.shape
        dy = dy.to(torch.bfloat16).contiguous()
        dx = torch.empty(N, D, H, W, C, dtype=torch.bfloat16, device=dy.device)
        _native.kernels().upsample2x(dy.data_ptr(), dx.data_ptr(), N, D, H, W, C, 1, _native.stream(dy))
        return dx


def upsample2x(x5: torch.Tensor) -> torch.Tensor:
    """[N, D, H, W, C] -> [N, 2D, 2H, 2W, C], nearest neighbour."""
    if _native.use_native(x5) and x5.shape[-1] % 8 == 0:
        return Upsample2xFn.apply(x5)
    n, d, h, w, c = x5.shape
    return x5.reshape(n, d, 1, h, 1, w, 1, c).expand(n, d, 2, h, 2, w, 2, c).reshape(n, 2 * d, 2 * h, 2 * w, c)
