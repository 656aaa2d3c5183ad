"""Differentiable ops over channels-last activations.

GPU tensors run the hand-written gfx950 HIP kernels (``csrc/kernels``); CPU
tensors run the PyTorch reference twins in :mod:`.reference`.
"""
from .bn import batchnorm_act, batchnorm_act_pool
from .conv import conv, depthwise_conv
from .elementwise import activation, add, concat, dropout, multiply, zero_pad
from .linear import linear
from .loss import softmax_xent
from .optim import FlatAdam, FlatSGD
from .pool import global_avg_pool, pool
from .spec import ConvSpec, PoolSpec, to5d_shape

__all__ = [
    "batchnorm_act", "batchnorm_act_pool", "conv", "depthwise_conv", "activation", "add", "concat", "dropout", "multiply",
    "zero_pad", "linear", "softmax_xent", "FlatAdam", "FlatSGD", "global_avg_pool", "pool", "ConvSpec",
    "PoolSpec", "to5d_shape",
]
