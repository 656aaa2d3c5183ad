"""Max / average / global-average pooling (reference ``model/input.py:193-243``:
MaxPooling2D / AveragePooling2D with the kernel clamped to <= 3 and padding
forced to ``same``, and GlobalAveragePooling2D) plus the 3-D MaxPool3d of
FeatureNet-3D.  GPU: ``pool_fwd`` / ``pool_bwd`` in ``bn_pool.hip``."""
from __future__ import annotations

import torch

from .. import _native
from . import reference as ref
from .spec import PoolSpec


class PoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x5, pspec: PoolSpec, is_max: bool, count_pad: bool):
        out = torch.empty(pspec.out_shape5, dtype=torch.bfloat16, device=x5.device)
        _native.kernels().pool_fwd(x5.data_ptr(), out.data_ptr(), 0, 0, pspec.geom17(), int(is_max), int(count_pad),
                                   0, _native.stream(x5), [x5.numel(), out.numel()])
        ctx.save_for_backward(x5)
        ctx.pspec, ctx.is_max, ctx.count_pad = pspec, is_max, count_pad
        return out

    @staticmethod
    def backward(ctx, dout):
        (x5,) = ctx.saved_tensors
        dx = torch.empty_like(x5)
        dout = dout.contiguous().to(torch.bfloat16)
        _native.kernels().pool_bwd(dout.data_ptr(), x5.data_ptr(), dx.data_ptr(), 0, 0, ctx.pspec.geom17(),
                                   int(ctx.is_max), int(ctx.count_pad), 0, _native.stream(x5),
                                   [min(x5.numel(), dx.numel()), dout.numel()])
        return dx, None, None, None


def pool(x5: torch.Tensor, pspec: PoolSpec, kind: str = "max", count_pad: bool = False) -> torch.Tensor:
    if _native.use_native(x5):
        return PoolFn.apply(x5.to(torch.bfloat16).contiguous(), pspec, kind == "max", count_pad)
    return ref.pool(x5, pspec, kind, count_pad)


def global_avg_pool(x5: torch.Tensor) -> torch.Tensor:
    """[N,D,H,W,C] -> [N,C] (Keras GlobalAveragePooling)."""
    N, D, H, W, C = x5.shape
    spec = PoolSpec.make(x5.shape, (D, H, W), (D, H, W), "valid")
    return pool(x5, spec, "avg").reshape(N, C)
