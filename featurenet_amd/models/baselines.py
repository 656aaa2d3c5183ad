"""Hand-written baseline CNNs (reference ``lenet5.py``, ``alexnet.py``,
``squeezenet.py``), on the same native layers as the NAS candidates.

They are the comparison points the reference uses for "template vs
hand-written" parity (``full_lenet5.py:48-54``, ``plots/plotter.py:128-169``).
Inputs are channels-last ``[N, H, W, C]``; outputs are logits (softmax lives in
the loss).

Reference quirk kept behind ``compat``: SqueezeNet declares
``data_format="channels_first"`` on NHWC data (``squeezenet.py:20-152``), so a
32x32x3 CIFAR image is treated as 32 channels of 32x3 pixels; with
``compat=True`` the model is built that way and reproduces the published
parameter count (876,970, ``squeezenet.py:231``); ``compat=False`` (default)
builds the intended 3-channel network.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .layers import BatchNorm, Conv, Dense, Pool


def _pool(k, s, kind="max"):
    return Pool((1, k, k), (1, s, s), "valid", kind)


class LeNet5(nn.Module):
    """``lenet5.py:8-20``: conv6 5x5 same tanh, avgpool 2/1, conv16 5x5 tanh, avgpool 2/2,
    conv120 5x5 tanh, dense84 tanh, dense n."""

    def __init__(self, input_shape=(28, 28, 1), num_classes: int = 10):
        super().__init__()
        H, W, C = input_shape
        self.c1 = Conv(C, 6, (1, 5, 5), 1, "same", act="tanh")
        self.p1 = _pool(2, 1, "avg")
        self.c2 = Conv(6, 16, (1, 5, 5), 1, "valid", act="tanh")
        self.p2 = _pool(2, 2, "avg")
        self.c3 = Conv(16, 120, (1, 5, 5), 1, "valid", act="tanh")
        h = ((H - 1 - 4) // 2) - 4
        w = ((W - 1 - 4) // 2) - 4
        self.fc1 = Dense(h * w * 120, 84, act="tanh")
        self.fc2 = Dense(84, num_classes)

    def forward(self, x):
        y = self.c3(self.p2(self.c2(self.p1(self.c1(x)))))
        y = self.fc1(y.reshape(len(y), -1))
        return self.fc2(y, out_fp32=True) if y.is_cuda else self.fc2(y).float()


class AlexNet(nn.Module):
    """``alexnet.py:8-75``: 5 conv (+ReLU, pools, BN) and 3 dense (+ReLU, dropout 0.4, BN)."""

    def __init__(self, input_shape=(224, 224, 3), num_classes: int = 10, dropout: float = 0.4):
        super().__init__()
        H, W, C = input_shape
        cfg = [(96, 11, 4, True), (256, 11, 1, True), (384, 3, 1, False), (384, 3, 1, False), (256, 3, 1, True)]
        self.features = nn.ModuleList()
        cin = C
        for cout, k, s, pool in cfg:
            self.features.append(Conv(cin, cout, (1, k, k), (1, s, s), "valid", act="relu"))
            H, W = (H - k) // s + 1, (W - k) // s + 1
            if pool:
                self.features.append(_pool(2, 2))
                H, W = H // 2, W // 2
            self.features.append(BatchNorm(cout))
            cin = cout
        if min(H, W) < 1:
            raise ValueError("input too small for AlexNet")
        self.dropout = dropout
        self.fcs = nn.ModuleList([Dense(H * W * cin, 4096, act="relu"), Dense(4096, 4096, act="relu"),
                                  Dense(4096, 1000, act="relu")])
        self.bns = nn.ModuleList([BatchNorm(4096), BatchNorm(4096), BatchNorm(1000)])
        self.head = Dense(1000, num_classes)

    def forward(self, x):
        for m in self.features:
            x = m(x)
        x = x.reshape(len(x), -1)
        for fc, bn in zip(self.fcs, self.bns):
            x = bn(ops.dropout(fc(x), self.dropout, self.training))
        return self.head(x, out_fp32=True) if x.is_cuda else self.head(x).float()


class Fire(nn.Module):
    def __init__(self, cin, squeeze, expand):
        super().__init__()
        self.sq = Conv(cin, squeeze, (1, 1, 1), 1, "same", act="relu")
        self.e1 = Conv(squeeze, expand, (1, 1, 1), 1, "same", act="relu")
        self.e3 = Conv(squeeze, expand, (1, 3, 3), 1, "same", act="relu")

    def forward(self, x):
        s = self.sq(x)
        return ops.concat([self.e1(s), self.e3(s)], -1)


class SqueezeNet(nn.Module):
    """SqueezeNet v1 (``squeezenet.py:17-156``): conv1 7x7/2 96, 8 fire modules with
    1x1 stride-2 'maxpools', dropout 0.5, conv10 1x1 (ReLU), global average pool."""

    FIRES = [(16, 64), (16, 64), (32, 128), "pool", (32, 128), (48, 192), (48, 192), (64, 256), "pool", (64, 256)]

    def __init__(self, input_shape=(32, 32, 3), num_classes: int = 10, compat: bool = False):
        super().__init__()
        self.compat = compat
        H, W, C = input_shape
        cin = H if compat else C         # channels_first on NHWC: the first spatial axis becomes channels
        self.conv1 = Conv(cin, 96, (1, 7, 7), (1, 2, 2), "same", act="relu")
        self.mods = nn.ModuleList()
        self.pool = _pool(1, 2)          # MaxPooling2D(pool_size=1, strides=2): a strided subsample
        c = 96
        for f in ["pool"] + self.FIRES:
            if f == "pool":
                self.mods.append(self.pool)
            else:
                self.mods.append(Fire(c, *f))
                c = 2 * f[1]
        self.conv10 = Conv(c, num_classes, (1, 1, 1), 1, "valid", act="relu")

    def forward(self, x):
        if self.compat:
            x = x.permute(0, 2, 3, 1)    # [N, H, W, C] seen as [N, C=H, W, C]: channels-last view of that
        x = self.conv1(x)
        for i, m in enumerate(self.mods):
            x = m(x)
        x = ops.dropout(x, 0.5, self.training)
        x = self.conv10(x)
        x5 = x.reshape(ops.to5d_shape(x.shape))
        return ops.global_avg_pool(x5).float() if x.is_cuda else x5.float().mean((1, 2, 3))


BASELINES = {"lenet": LeNet5, "lenet5-handwritten": LeNet5, "alexnet": AlexNet, "squeezenet": SqueezeNet}


def count_params(m: nn.Module) -> int:
    """Keras ``count_params``: trainable + BN moving statistics."""
    n = sum(p.numel() for p in m.parameters())
    n += sum(b.numel() for k, b in m.named_buffers() if k.endswith(("running_mean", "running_var")))
    return n


def build_baseline(name: str, input_shape, num_classes: int, **kw) -> nn.Module:
    return BASELINES[name.lower()](tuple(input_shape), num_classes, **kw)


__all__ = ["LeNet5", "AlexNet", "SqueezeNet", "Fire", "BASELINES", "build_baseline", "count_params"]
_ = torch
