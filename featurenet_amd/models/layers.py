"""Layer modules over channels-last activations.

Parameters are fp32 masters; the native ops cast to bf16 at the point of
use.  Initialisers follow the Keras 2.2 defaults the reference relied on
(``glorot_uniform`` kernels, zero biases, BN gamma=1 / beta=0) unless a
model asks otherwise.
"""
from __future__ import annotations

import math

import torch
from torch import nn

from .. import ops
from ..ops.spec import ConvSpec, PoolSpec, _triple, to5d_shape


def glorot_uniform_(w: torch.Tensor, fan_in: int, fan_out: int, gen: torch.Generator | None = None) -> torch.Tensor:
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    with torch.no_grad():
        return w.uniform_(-lim, lim, generator=gen)


def he_normal_(w: torch.Tensor, fan_in: int, gen: torch.Generator | None = None) -> torch.Tensor:
    with torch.no_grad():
        return w.normal_(0.0, math.sqrt(2.0 / fan_in), generator=gen)


class Conv(nn.Module):
    """N-d convolution (1/2/3-D, channels-last) with optional fused BN, activation and pooling.

    GPU fusion: conv epilogue emits BN statistics, BN+act is applied inside the
    pooling kernel when a pool follows (the normalised tensor never hits HBM).
    In eval mode BN is folded into the conv weights/bias and BN+act run in the
    conv epilogue.
    """

    def __init__(self, cin: int, cout: int, kernel, stride=1, padding="valid", dilation=1, bn: bool = False,
                 act=None, pool=None, pool_stride=None, pool_kind: str = "max", pool_padding="valid",
                 bias: bool | None = None, init: str = "glorot", bn_momentum: float = 0.1, bn_eps: float = 1e-5):
        super().__init__()
        self.cin, self.cout = cin, cout
        self.kernel = _triple(kernel)
        self.stride, self.padding, self.dilation = stride, padding, dilation
        self.act = act
        self.bn = bn
        self.pool = None if pool is None else _triple(pool)
        self.pool_stride, self.pool_kind, self.pool_padding = pool_stride, pool_kind, pool_padding
        KD, KH, KW = self.kernel
        self.weight = nn.Parameter(torch.empty(cout, KD, KH, KW, cin))
        fan_in, fan_out = cin * KD * KH * KW, cout * KD * KH * KW
        if init == "he":
            he_normal_(self.weight, fan_in)
        else:
            glorot_uniform_(self.weight, fan_in, fan_out)
        use_bias = (not bn) if bias is None else bias
        self.bias = nn.Parameter(torch.zeros(cout)) if use_bias else None
        if bn:
            self.gamma = nn.Parameter(torch.ones(cout))
            self.beta = nn.Parameter(torch.zeros(cout))
            self.register_buffer("running_mean", torch.zeros(cout))
            self.register_buffer("running_var", torch.ones(cout))
            self.bn_momentum, self.bn_eps = bn_momentum, bn_eps
        self._spec_cache: dict = {}

    def specs(self, shape5):
        s = self._spec_cache.get(shape5)
        if s is None:
            cs = ConvSpec.make(shape5, self.cout, self.kernel, self.stride, self.padding, self.dilation,
                               extra=getattr(self, "extra_pad", (0, 0, 0)))
            ps = None
            if self.pool is not None:
                ps = PoolSpec.make(cs.out_shape5, self.pool, self.pool_stride, self.pool_padding)
            s = (cs, ps)
            self._spec_cache[shape5] = s
        return s

    def forward(self, x: torch.Tensor, conv_next: bool = False) -> torch.Tensor:
        """``conv_next``: the output goes to one following Conv and nowhere else, so a BN + act
        output may be left to that conv's forward kernel to write (ops/bn.py ``batchnorm_act``)."""
        in_shape = x.shape
        x5 = x.reshape(to5d_shape(in_shape))
        cs, ps = self.specs(tuple(x5.shape))
        if self.bn and not self.training:
            # inference: BN folded into the conv (w * gamma/sigma, beta - mean * gamma/sigma), so
            # BN + act run in the conv epilogue -- no statistics, no separate normalise pass
            scale = self.gamma * torch.rsqrt(self.running_var + self.bn_eps)
            w = self.weight * scale.view(-1, 1, 1, 1, 1)
            b = self.beta - self.running_mean * scale
            out = ops.conv(x5, w, b, cs, self.act)
            if ps is not None:
                out = ops.pool(out, ps, self.pool_kind)
        elif self.bn:
            y, slab = ops.conv(x5, self.weight, None, cs, None, want_stats=True)
            if ps is not None:
                out = ops.batchnorm_act_pool(y, self.gamma, self.beta, self.running_mean, self.running_var,
                                             self.training, ps, self.pool_kind, self.bn_momentum, self.bn_eps,
                                             self.act, stats_slab=slab)
            else:
                out = ops.batchnorm_act(y, self.gamma, self.beta, self.running_mean, self.running_var,
                                        self.training, self.bn_momentum, self.bn_eps, self.act, stats_slab=slab,
                                        conv_next=conv_next)
        else:
            out = ops.conv(x5, self.weight, self.bias, cs, self.act)
            if ps is not None:
                out = ops.pool(out, ps, self.pool_kind)
        # restore the caller's rank
        n, d, h, w, c = out.shape
        if len(in_shape) == 4:
            return out.reshape(n, h, w, c)
        if len(in_shape) == 3:
            return out.reshape(n, w, c)
        return out

    def flops(self, shape5) -> int:
        cs, _ = self.specs(tuple(shape5))
        return cs.flops()


class Dense(nn.Module):
    """Dense layer applied on the last axis (Keras semantics for any rank)."""

    def __init__(self, fin: int, fout: int, act=None, bias: bool = True, init: str = "glorot"):
        super().__init__()
        self.fin, self.fout, self.act = fin, fout, act
        self.weight = nn.Parameter(torch.empty(fout, fin))
        if init == "he":
            he_normal_(self.weight, fin)
        else:
            glorot_uniform_(self.weight, fin, fout)
        self.bias = nn.Parameter(torch.zeros(fout)) if bias else None

    def forward(self, x: torch.Tensor, out_fp32: bool = False) -> torch.Tensor:
        return ops.linear(x, self.weight, self.bias, self.act, out_fp32=out_fp32)


class BatchNorm(nn.Module):
    """Standalone BN(+act) over the last (channel) axis."""

    def __init__(self, channels: int, act=None, momentum: float = 0.1, eps: float = 1e-5):
        super().__init__()
        self.act = act
        self.gamma = nn.Parameter(torch.ones(channels))
        self.beta = nn.Parameter(torch.zeros(channels))
        self.register_buffer("running_mean", torch.zeros(channels))
        self.register_buffer("running_var", torch.ones(channels))
        self.momentum, self.eps = momentum, eps

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        shape = x.shape
        x5 = x.reshape(-1, 1, 1, 1, shape[-1])
        out = ops.batchnorm_act(x5, self.gamma, self.beta, self.running_mean, self.running_var, self.training,
                                self.momentum, self.eps, self.act)
        return out.reshape(shape)


class Pool(nn.Module):
    def __init__(self, kernel, stride=None, padding="valid", kind: str = "max"):
        super().__init__()
        self.kernel, self.stride, self.padding, self.kind = _triple(kernel), stride, padding, kind

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        shape = x.shape
        x5 = x.reshape(to5d_shape(shape))
        ps = PoolSpec.make(tuple(x5.shape), self.kernel, self.stride, self.padding)
        out = ops.pool(x5, ps, self.kind)
        n, d, h, w, c = out.shape
        if len(shape) == 4:
            return out.reshape(n, h, w, c)
        if len(shape) == 3:
            return out.reshape(n, w, c)
        return out


class DepthwiseConv(nn.Module):
    """Depthwise convolution (Keras ``DepthwiseConv2D``, depth_multiplier ``mult``)."""

    def __init__(self, cin: int, kernel, stride=1, padding="same", act=None, mult: int = 1, bias: bool = True):
        super().__init__()
        self.cin, self.mult, self.act = cin, mult, act
        self.kernel = _triple(kernel)
        self.stride, self.padding = stride, padding
        KD, KH, KW = self.kernel
        self.weight = nn.Parameter(torch.empty(cin * mult, KD, KH, KW, 1))
        glorot_uniform_(self.weight, KD * KH * KW, KD * KH * KW * mult)
        self.bias = nn.Parameter(torch.zeros(cin * mult)) if bias else None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        shape = x.shape
        x5 = x.reshape(to5d_shape(shape))
        cs = ConvSpec.make(tuple(x5.shape), self.cin * self.mult, self.kernel, self.stride, self.padding)
        out = ops.depthwise_conv(x5, self.weight, self.bias, cs, self.mult, self.act)
        n, d, h, w, c = out.shape
        if len(shape) == 4:
            return out.reshape(n, h, w, c)
        if len(shape) == 3:
            return out.reshape(n, w, c)
        return out


class SeparableConv(nn.Module):
    """Keras ``SeparableConv1D/2D``: depthwise (no bias) -> pointwise 1x1 (bias) -> activation."""

    def __init__(self, cin: int, cout: int, kernel, stride=1, padding="same", act=None):
        super().__init__()
        self.depthwise = DepthwiseConv(cin, kernel, stride, padding, None, 1, bias=False)
        self.pointwise = Conv(cin, cout, 1, 1, "valid", act=act, bias=True)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.pointwise(self.depthwise(x))


class AxisBatchNorm(nn.Module):
    """BatchNorm over an arbitrary axis (the reference forces ``axis=1``,
    ``model/operation.py:142``; on NHWC tensors that normalises per image row)."""

    def __init__(self, channels: int, axis: int = -1, act=None, momentum: float = 0.01, eps: float = 1e-3):
        super().__init__()
        self.axis = axis
        self.bn = BatchNorm(channels, act, momentum, eps)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        ax = self.axis if self.axis >= 0 else x.dim() + self.axis
        if ax == x.dim() - 1:
            return self.bn(x)
        xt = x.movedim(ax, -1).contiguous()
        return self.bn(xt).movedim(-1, ax).contiguous()
