"""Geometry specs shared by the native kernels and the reference path.

All activations are channels-last: 3-D ``[N, D, H, W, C]``, 2-D
``[N, H, W, C]``, 1-D ``[N, W, C]``.  Internally every op works on the 5-D view
(2-D = ``D == 1``; 1-D = ``D == H == 1``).  Convolution weights are stored
``[Cout, KD, KH, KW, Cin]`` so a row of the GEMM ``B`` operand (one output
channel) is contiguous in the reduction index ``k = ((kd*KH + kh)*KW + kw)*Cin + ci``.

Padding follows Keras semantics (reference ``model/input.py:250``: every conv
and pooling layer is forced to ``padding="same"``): "same" pads
``max((out-1)*s + (k-1)*d + 1 - in, 0)`` elements, ``total // 2`` before and the
rest after; "valid" pads nothing.  Only the leading pad is needed by the
kernels -- taps that fall past the end read zero.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Sequence


def _triple(v, fill=1) -> tuple[int, int, int]:
    if isinstance(v, int):
        return (v, v, v)
    v = tuple(int(a) for a in v)
    while len(v) < 3:
        v = (fill,) + v
    return v  # type: ignore[return-value]


def same_pad(inp: int, k: int, s: int, d: int = 1) -> tuple[int, int]:
    out = -(-inp // s)
    total = max((out - 1) * s + (k - 1) * d + 1 - inp, 0)
    return total // 2, total - total // 2


def out_size(inp: int, k: int, s: int, pad_lo: int, pad_hi: int, d: int = 1) -> int:
    return (inp + pad_lo + pad_hi - d * (k - 1) - 1) // s + 1


def to5d_shape(shape: Sequence[int]) -> tuple[int, int, int, int, int]:
    """Shape of the 5-D channels-last view of a 3/4/5-D activation."""
    if len(shape) == 5:
        return tuple(shape)  # type: ignore[return-value]
    if len(shape) == 4:
        n, h, w, c = shape
        return (n, 1, h, w, c)
    if len(shape) == 3:
        n, w, c = shape
        return (n, 1, 1, w, c)
    raise ValueError(f"expected a 3-, 4- or 5-D channels-last tensor, got shape {tuple(shape)}")


@dataclass(frozen=True)
class ConvSpec:
    N: int
    D: int
    H: int
    W: int
    C: int
    K: int                      # output channels
    KD: int
    KH: int
    KW: int
    sd: int = 1
    sh: int = 1
    sw: int = 1
    pd: int = 0                 # leading pads
    ph: int = 0
    pw: int = 0
    dd: int = 1
    dh: int = 1
    dw: int = 1
    OD: int = 0
    OH: int = 0
    OW: int = 0

    @staticmethod
    def make(x_shape5, cout: int, kernel, stride=1, padding="valid", dilation=1, extra=(0, 0, 0)) -> "ConvSpec":
        """``extra``: zero padding (per side, per dim) folded in from a preceding ZeroPadding
        layer: the conv behaves as on the input padded by it, then padded by ``padding``."""
        N, D, H, W, C = x_shape5
        if any(extra):
            pe = ConvSpec.make((N, D + 2 * extra[0], H + 2 * extra[1], W + 2 * extra[2], C), cout, kernel, stride,
                               padding, dilation)
            return ConvSpec(N, D, H, W, C, cout, pe.KD, pe.KH, pe.KW, pe.sd, pe.sh, pe.sw, pe.pd + extra[0],
                            pe.ph + extra[1], pe.pw + extra[2], pe.dd, pe.dh, pe.dw, pe.OD, pe.OH, pe.OW)
        KD, KH, KW = _triple(kernel)
        sd, sh, sw = _triple(stride)
        dd, dh, dw = _triple(dilation)
        dims = []
        for inp, k, s, d in ((D, KD, sd, dd), (H, KH, sh, dh), (W, KW, sw, dw)):
            if padding == "same":
                lo, hi = same_pad(inp, k, s, d)
            elif padding == "valid":
                lo, hi = 0, 0
            else:
                p = _triple(padding, 0)[len(dims)]
                lo, hi = p, p
            dims.append((lo, out_size(inp, k, s, lo, hi, d)))
        (pd, OD), (ph, OH), (pw, OW) = dims
        if min(OD, OH, OW) <= 0:
            raise ValueError(f"conv produces empty output: in={x_shape5} k={(KD, KH, KW)} s={(sd, sh, sw)}")
        return ConvSpec(N, D, H, W, C, cout, KD, KH, KW, sd, sh, sw, pd, ph, pw, dd, dh, dw, OD, OH, OW)

    @property
    def taps(self) -> int:
        return self.KD * self.KH * self.KW

    @property
    def kdim(self) -> int:
        return self.taps * self.C

    @property
    def M(self) -> int:
        return self.N * self.OD * self.OH * self.OW

    @property
    def out_shape5(self) -> tuple[int, int, int, int, int]:
        return (self.N, self.OD, self.OH, self.OW, self.K)

    @property
    def pads_hi(self) -> tuple[int, int, int]:
        """Trailing pads implied by the output size."""
        res = []
        for inp, k, s, d, lo, o in (
            (self.D, self.KD, self.sd, self.dd, self.pd, self.OD),
            (self.H, self.KH, self.sh, self.dh, self.ph, self.OH),
            (self.W, self.KW, self.sw, self.dw, self.pw, self.OW),
        ):
            res.append(max((o - 1) * s + (k - 1) * d + 1 - inp - lo, 0))
        return tuple(res)  # type: ignore[return-value]

    def flops(self) -> int:
        return 2 * self.M * self.K * self.kdim


@dataclass(frozen=True)
class PoolSpec:
    N: int
    D: int
    H: int
    W: int
    C: int
    KD: int
    KH: int
    KW: int
    sd: int
    sh: int
    sw: int
    pd: int
    ph: int
    pw: int
    OD: int
    OH: int
    OW: int

    @staticmethod
    def make(x_shape5, kernel, stride=None, padding="valid") -> "PoolSpec":
        N, D, H, W, C = x_shape5
        KD, KH, KW = _triple(kernel)
        if stride is None:
            stride = (KD, KH, KW)
        sd, sh, sw = _triple(stride)
        dims = []
        for inp, k, s in ((D, KD, sd), (H, KH, sh), (W, KW, sw)):
            if padding == "same":
                lo, hi = same_pad(inp, k, s)
            else:
                lo, hi = 0, 0
            dims.append((lo, out_size(inp, k, s, lo, hi)))
        (pd, OD), (ph, OH), (pw, OW) = dims
        if min(OD, OH, OW) <= 0:
            raise ValueError(f"pool produces empty output: in={x_shape5} k={(KD, KH, KW)}")
        return PoolSpec(N, D, H, W, C, KD, KH, KW, sd, sh, sw, pd, ph, pw, OD, OH, OW)

    @property
    def out_shape5(self):
        return (self.N, self.OD, self.OH, self.OW, self.C)

    def geom17(self) -> list[int]:
        return [self.N, self.D, self.H, self.W, self.C, self.OD, self.OH, self.OW, self.KD, self.KH, self.KW,
                self.sd, self.sh, self.sw, self.pd, self.ph, self.pw]


ACT_CODES = {None: 0, "none": 0, "linear": 0, "relu": 1, "tanh": 2, "sigmoid": 3}


def act_code(act) -> int:
    if act not in ACT_CODES:
        raise ValueError(f"activation {act!r} has no fused kernel form")
    return ACT_CODES[act]
