"""PyTorch reference implementations (the numerical oracle / CPU path).

Every native op in :mod:`featurenet_amd.ops` has a reference twin here with
the same channels-last calling convention.  CPU tensors run these directly
(BASELINE.json config 1: the CPU reference path); the kernel tests compare
the HIP kernels against them in fp32.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .spec import ConvSpec, PoolSpec


def to_ncdhw(x5: torch.Tensor) -> torch.Tensor:
    return x5.permute(0, 4, 1, 2, 3)


def to_ndhwc(x: torch.Tensor) -> torch.Tensor:
    return x.permute(0, 2, 3, 4, 1)


def activation(x: torch.Tensor, act) -> torch.Tensor:
    if act in (None, "none", "linear"):
        return x
    if act == "relu":
        return F.relu(x)
    if act == "tanh":
        return torch.tanh(x)
    if act == "sigmoid":
        return torch.sigmoid(x)
    if act == "softmax":
        return torch.softmax(x, dim=-1)
    raise ValueError(f"unknown activation {act!r}")


def conv(x5: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None, spec: ConvSpec, act=None) -> torch.Tensor:
    """x5 [N,D,H,W,C], w [K,KD,KH,KW,C] -> [N,OD,OH,OW,K]."""
    xin = to_ncdhw(x5)
    hd, hh, hw = spec.pads_hi
    if spec.pd or spec.ph or spec.pw or hd or hh or hw:
        xin = F.pad(xin, (spec.pw, hw, spec.ph, hh, spec.pd, hd))
    y = F.conv3d(xin, w.permute(0, 4, 1, 2, 3), b, stride=(spec.sd, spec.sh, spec.sw),
                 dilation=(spec.dd, spec.dh, spec.dw))
    y = y[:, :, : spec.OD, : spec.OH, : spec.OW]
    return activation(to_ndhwc(y), act)


def depthwise_conv(x5: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None, spec: ConvSpec, mult: int = 1,
                   act=None) -> torch.Tensor:
    """Depthwise: w [C*mult, KD, KH, KW, 1]."""
    xin = to_ncdhw(x5)
    hd, hh, hw = spec.pads_hi
    xin = F.pad(xin, (spec.pw, hw, spec.ph, hh, spec.pd, hd))
    y = F.conv3d(xin, w.permute(0, 4, 1, 2, 3), b, stride=(spec.sd, spec.sh, spec.sw),
                 dilation=(spec.dd, spec.dh, spec.dw), groups=spec.C)
    y = y[:, :, : spec.OD, : spec.OH, : spec.OW]
    return activation(to_ndhwc(y), act)


def batchnorm_act(y5: torch.Tensor, gamma, beta, running_mean, running_var, training: bool, momentum: float,
                  eps: float, act=None) -> torch.Tensor:
    C = y5.shape[-1]
    flat = y5.reshape(-1, C)
    z = F.batch_norm(flat, running_mean, running_var, gamma, beta, training, momentum, eps)
    return activation(z, act).reshape(y5.shape)


def pool(x5: torch.Tensor, spec: PoolSpec, kind: str = "max", count_pad: bool = False) -> torch.Tensor:
    xin = to_ncdhw(x5)
    k = (spec.KD, spec.KH, spec.KW)
    s = (spec.sd, spec.sh, spec.sw)
    hd = max((spec.OD - 1) * spec.sd + spec.KD - spec.D - spec.pd, 0)
    hh = max((spec.OH - 1) * spec.sh + spec.KH - spec.H - spec.ph, 0)
    hw = max((spec.OW - 1) * spec.sw + spec.KW - spec.W - spec.pw, 0)
    pads = (spec.pw, hw, spec.ph, hh, spec.pd, hd)
    if kind == "max":
        if any(pads):
            xin = F.pad(xin, pads, value=float("-inf"))
        y = F.max_pool3d(xin, k, s)
    else:
        if any(pads):
            ones = torch.ones_like(xin[:, :1])
            num = F.avg_pool3d(F.pad(xin, pads), k, s, divisor_override=1)
            if count_pad:
                den = torch.full_like(num[:, :1], float(spec.KD * spec.KH * spec.KW))
            else:
                den = F.avg_pool3d(F.pad(ones, pads), k, s, divisor_override=1)
            y = num / den
        else:
            y = F.avg_pool3d(xin, k, s)
    y = y[:, :, : spec.OD, : spec.OH, : spec.OW]
    return to_ndhwc(y)


def softmax_xent(logits: torch.Tensor, labels: torch.Tensor, smoothing: float = 0.0) -> torch.Tensor:
    lg = logits if logits.dtype == torch.float64 else logits.float()   # >= fp32 (fp64 kept for gradcheck)
    return F.cross_entropy(lg, labels, label_smoothing=smoothing)
