"""Activation, dropout and the branch-combination ops.

Reference parity: ``Activation`` (``model/operation.py:152-165``), ``Dropout``
(``:103-114``), ``Add`` / ``Concatenate`` / ``Multiply`` (``:214-248``),
``ZeroPadding2D`` (``:116-137``), ``K.zeros`` (``model/input.py:159-165``).

GPU: activation fwd/bwd and dropout (counter-hash mask regenerated in
backward, never stored) are native kernels, and so are add / multiply (fused
multiply backward), two-way concat (each input written into its column range)
and zero padding (border + interior in one pass) -- ``csrc/kernels/combine.hip``.
A ZeroPadding whose only consumer is a convolution is folded into that
convolution's padding by the IR compiler instead (no padded tensor at all).
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


def _native_pair(a: torch.Tensor, b: torch.Tensor) -> bool:
    return _native.use_native(a) and a.shape == b.shape and a.is_cuda and b.is_cuda


class BinaryFn(torch.autograd.Function):
    """out = a + b (op 0) or a * b (op 1), bf16, one pass (``ew_binary``)."""

    @staticmethod
    def forward(ctx, a, b, op: int):
        ab, bb = a.to(torch.bfloat16).contiguous(), b.to(torch.bfloat16).contiguous()
        out = torch.empty_like(ab)
        _native.kernels().ew_binary(ab.data_ptr(), bb.data_ptr(), out.data_ptr(), ab.numel(), op, _native.stream(ab))
        ctx.op = op
        if op == 1:
            ctx.save_for_backward(ab, bb)
        return out

    @staticmethod
    def backward(ctx, g):
        if ctx.op == 0:
            return g, g, None
        ab, bb = ctx.saved_tensors
        g = g.to(torch.bfloat16).contiguous()
        da, db = torch.empty_like(g), torch.empty_like(g)
        _native.kernels().ew_mul_bwd(g.data_ptr(), ab.data_ptr(), bb.data_ptr(), da.data_ptr(), db.data_ptr(),
                                     g.numel(), _native.stream(g))
        return da, db, None


def add(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Keras ``Add`` of two branches (native one-pass kernel on GPU)."""
    if _native_pair(a, b):
        return BinaryFn.apply(a, b, 0)
    return a + b


def multiply(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Keras ``Multiply`` (native forward and one-pass fused backward on GPU)."""
    if _native_pair(a, b):
        return BinaryFn.apply(a, b, 1)
    return a * b


class Concat2Fn(torch.autograd.Function):
    """Two tensors joined along ``axis``: each input is written into its column range of the
    output (``concat2``); the backward splits the gradient with the same kernel."""

    @staticmethod
    def forward(ctx, a, b, axis: int):
        ab, bb = a.to(torch.bfloat16).contiguous(), b.to(torch.bfloat16).contiguous()
        shape = list(ab.shape)
        shape[axis] += bb.shape[axis]
        out = torch.empty(shape, dtype=torch.bfloat16, device=ab.device)
        outer = 1
        for d in ab.shape[:axis]:
            outer *= d
        ia, ib = ab.numel() // outer, bb.numel() // outer
        _native.kernels().concat2(ab.data_ptr(), bb.data_ptr(), out.data_ptr(), outer, ia, ib, 0, _native.stream(ab))
        ctx.meta = (ab.shape, bb.shape, outer, ia, ib)
        return out

    @staticmethod
    def backward(ctx, g):
        sa, sb, outer, ia, ib = ctx.meta
        g = g.to(torch.bfloat16).contiguous()
        da = torch.empty(sa, dtype=torch.bfloat16, device=g.device)
        db = torch.empty(sb, dtype=torch.bfloat16, device=g.device)
        _native.kernels().concat2(da.data_ptr(), db.data_ptr(), g.data_ptr(), outer, ia, ib, 1, _native.stream(g))
        return da, db, None


def concat(tensors, axis: int) -> torch.Tensor:
    tensors = list(tensors)
    if len(tensors) == 2 and _native.use_native(tensors[0]) and tensors[0].is_cuda and tensors[1].is_cuda:
        a, b = tensors
        ax = axis % a.dim()
        if a.dim() == b.dim() and all(a.shape[i] == b.shape[i] for i in range(a.dim()) if i != ax):
            return Concat2Fn.apply(a, b, ax)
    return torch.cat(tensors, dim=axis)


class Pad3Fn(torch.autograd.Function):
    """Zero padding of a channels-last [N, D, H, W, C] grid (``pad3``: border and interior in
    one pass; the backward crops the interior)."""

    @staticmethod
    def forward(ctx, x5, pads):
        xb = x5.to(torch.bfloat16).contiguous()
        N, D, H, W, C = xb.shape
        pd, ph, pw = pads
        out = torch.empty(N, D + 2 * pd, H + 2 * ph, W + 2 * pw, C, dtype=torch.bfloat16, device=xb.device)
        geom = [N, D, H, W, C, pd, ph, pw]
        _native.kernels().pad3(xb.data_ptr(), out.data_ptr(), geom, 0, _native.stream(xb))
        ctx.geom = geom
        return out

    @staticmethod
    def backward(ctx, g):
        N, D, H, W, C = ctx.geom[:5]
        g = g.to(torch.bfloat16).contiguous()
        dx = torch.empty(N, D, H, W, C, dtype=torch.bfloat16, device=g.device)
        _native.kernels().pad3(dx.data_ptr(), g.data_ptr(), ctx.geom, 1, _native.stream(g))
        return dx, None


def zero_pad(x5: torch.Tensor, pads) -> torch.Tensor:
    """Zero-pad spatial dims of a 5-D channels-last tensor; pads = (d, h, w) per side."""
    pd, ph, pw = pads
    if _native.use_native(x5) and x5.is_cuda and x5.dim() == 5:
        return Pad3Fn.apply(x5, (pd, ph, pw))
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
