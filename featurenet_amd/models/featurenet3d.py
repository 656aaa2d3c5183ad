"""FeatureNet-3D: the voxel machining-feature classifier (north-star workload).

Architecture (Zhang, Jaiswal & Rai, "FeatureNet: Machining feature
recognition based on 3D Convolution Neural Network", CAD 2018 -- recalled, not
present in the reference repository):

    64^3 x 1 occupancy grid
    Conv3d 32 @ 7^3, stride 2   -> 29^3   (BN + ReLU)
    Conv3d 32 @ 5^3             -> 25^3   (BN + ReLU)
    Conv3d 64 @ 4^3             -> 22^3   (BN + ReLU)
    Conv3d 64 @ 3^3             -> 20^3   (BN + ReLU + MaxPool3d 2^3 -> 10^3, fused)
    Dense 128 (ReLU)
    Dense 24 (softmax, fused into the loss)

All four convolutions run on the implicit-GEMM MFMA kernels; BN statistics
come out of the conv epilogue; conv4's BN+ReLU is applied inside the
MaxPool3d kernel.  The same class builds the tiny "16^3, 2-class" CPU
reference configuration and the per-voxel segmentation variant
(:class:`FeatureNet3DSeg`).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass

import torch
from torch import nn

from .. import ops
from ..ops import bn as bn_ops
from ..ops import subpixel
from ..ops.elementwise import upsample2x
from .layers import Conv, Dense


@dataclass
class FeatureNet3DConfig:
    input_size: int = 64
    in_channels: int = 1
    num_classes: int = 24
    widths: tuple = (32, 32, 64, 64)
    kernels: tuple = (7, 5, 4, 3)
    strides: tuple = (2, 1, 1, 1)
    pool: int = 2
    fc: int = 128
    bn: bool = True
    init: str = "he"

    def to_dict(self) -> dict:
        d = asdict(self)
        return {k: list(v) if isinstance(v, tuple) else v for k, v in d.items()}

    @staticmethod
    def from_dict(d: dict) -> "FeatureNet3DConfig":
        d = dict(d)
        for k in ("widths", "kernels", "strides"):
            if k in d:
                d[k] = tuple(d[k])
        return FeatureNet3DConfig(**d)

    @staticmethod
    def tiny() -> "FeatureNet3DConfig":
        """16^3-voxel 2-class tiny 3D-CNN (BASELINE.json config 1, CPU plumbing)."""
        return FeatureNet3DConfig(input_size=16, num_classes=2, widths=(8, 8, 16, 16), kernels=(3, 3, 3, 3),
                                  strides=(1, 1, 1, 1), pool=2, fc=32)


def _feature_shape(cfg: FeatureNet3DConfig) -> tuple[int, int]:
    s = cfg.input_size
    for k, st in zip(cfg.kernels, cfg.strides):
        s = (s - k) // st + 1
    s = s // cfg.pool
    if s <= 0:
        raise ValueError(f"FeatureNet-3D config collapses the {cfg.input_size}^3 input to nothing")
    return s, cfg.widths[-1]


class FeatureNet3D(nn.Module):
    def __init__(self, cfg: FeatureNet3DConfig | None = None):
        super().__init__()
        self.cfg = cfg = cfg or FeatureNet3DConfig()
        convs = []
        cin = cfg.in_channels
        n = len(cfg.widths)
        for i, (w, k, s) in enumerate(zip(cfg.widths, cfg.kernels, cfg.strides)):
            last = i == n - 1
            convs.append(Conv(cin, w, (k, k, k), (s, s, s), "valid", bn=cfg.bn, act="relu",
                              pool=(cfg.pool,) * 3 if last and cfg.pool > 1 else None, init=cfg.init))
            cin = w
        self.convs = nn.ModuleList(convs)
        sp, c = _feature_shape(cfg)
        self.flat_features = sp ** 3 * c
        self.fc1 = Dense(self.flat_features, cfg.fc, act="relu", init=cfg.init)
        self.fc2 = Dense(cfg.fc, cfg.num_classes, act=None)

    def features(self, x: torch.Tensor) -> torch.Tensor:
        if x.dim() == 4:  # [N, D, H, W] occupancy -> add channel axis
            x = x.unsqueeze(-1)
        n = len(self.convs)
        for i, c in enumerate(self.convs):
            # (each BN + ReLU output but the last feeds only the next conv: that conv's forward
            # kernel normalises its input halo itself and writes it, ops/bnfuse.py defer)
            x = c(x, conv_next=i < n - 1)
        return x

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x: [N, S, S, S, 1] (or [N, S, S, S]) -> fp32 logits [N, num_classes]."""
        # (no packs.pack_scope here: the three tile-stream packs in one launch measured neutral on
        # this step -- 4.633 vs 4.632 ms -- and the seg step slower, 19.05 vs 18.91 ms; NAS
        # candidates, with one 3-5 us pack per conv and direction, gain 2.5 %)
        f = self.features(x)
        f = f.reshape(f.shape[0], -1)
        h = self.fc1(f)
        return self.fc2(h, out_fp32=True)

    def train_flops_per_sample(self) -> int:
        """Analytic FLOPs of one training sample (fwd + dgrad + wgrad)."""
        cfg = self.cfg
        shape = (1, cfg.input_size, cfg.input_size, cfg.input_size, cfg.in_channels)
        fwd = 0
        bwd = 0
        for i, c in enumerate(self.convs):
            cs, ps = c.specs(shape)
            f = cs.flops()
            fwd += f
            bwd += f * (2 if i > 0 else 1)  # conv1 needs no dgrad (input has no grad)
            shape = ps.out_shape5 if ps is not None else cs.out_shape5
        fc = 2 * (self.flat_features * cfg.fc + cfg.fc * cfg.num_classes)
        return fwd + bwd + 3 * fc


class FeatureNet3DSeg(nn.Module):
    """Per-voxel multi-feature segmentation head (BASELINE.json config 4).

    Encoder = FeatureNet-3D convs with ``same`` padding (spatial size kept
    except for the stride-2 stem), decoder = nearest 2x upsample + 3^3 conv
    back to the input grid, 1x1x1 classifier producing per-voxel logits
    ``[N, S, S, S, num_classes]``.
    """

    def __init__(self, input_size: int = 64, in_channels: int = 1, num_classes: int = 25, widths=(32, 32, 64, 64)):
        super().__init__()
        self.input_size, self.num_classes = input_size, num_classes
        w0, w1, w2, w3 = widths
        self.enc = nn.ModuleList([
            Conv(in_channels, w0, (7, 7, 7), (2, 2, 2), "same", bn=True, act="relu", init="he"),
            Conv(w0, w1, (5, 5, 5), 1, "same", bn=True, act="relu", init="he"),
            Conv(w1, w2, (4, 4, 4), 1, "same", bn=True, act="relu", init="he"),
            Conv(w2, w3, (3, 3, 3), 1, "same", bn=True, act="relu", init="he"),
        ])
        self.dec = Conv(w3, w1, (3, 3, 3), 1, "same", bn=True, act="relu", init="he")
        self.head = Conv(w1, num_classes, (1, 1, 1), 1, "valid", bn=False, act=None, bias=True)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.dim() == 4:
            x = x.unsqueeze(-1)
        for i, c in enumerate(self.enc):
            x = c(x, conv_next=i < len(self.enc) - 1)
        return self._decode(x)

    def _decode(self, x: torch.Tensor) -> torch.Tensor:
        d, h = self.dec, self.head
        if self.training and subpixel.gpu_ok(x, d.cout, x.shape[-1]) and \
                bn_ops.fused_pointwise_ok(x, d.cout, h.cout, d.act):
            # training on the GPU: upsample + decoder conv as 8 parity-class 2^3 convs (3.4x
            # fewer FLOPs, the 2x-upsampled tensor never exists), the BN + ReLU inside the 1x1
            # head's kernels, backward through the shifted space-to-depth dy (ops/subpixel.py)
            return subpixel.decoder_head(x, d.weight, d.gamma, d.beta, d.running_mean, d.running_var, h.weight,
                                         h.bias, d.bn_momentum, d.bn_eps, d.act)
        x = upsample2x(x)                  # nearest x2 upsample on the channels-last grid
        if self.training and bn_ops.fused_pointwise_ok(x, d.cout, h.cout, d.act):
            # training on the GPU: the decoder's BN + ReLU run inside the 1x1 head's pointwise
            # kernels (forward and weight gradient), so its 64^3 x 32 output is never written
            cs, _ = d.specs(tuple(x.shape))
            y, slab = ops.conv(x, d.weight, None, cs, None, want_stats=True)
            return bn_ops.batchnorm_act_pointwise(y, d.gamma, d.beta, d.running_mean, d.running_var, h.weight, h.bias,
                                                  d.bn_momentum, d.bn_eps, d.act, stats_slab=slab)
        return h(d(x))  # [N, S, S, S, classes]

    def loss(self, x: torch.Tensor, labels: torch.Tensor, smoothing: float = 0.0, with_correct: bool = False):
        """Mean per-voxel softmax cross-entropy against ``labels`` [N, S, S, S] (+ the number of
        top-1 hits when ``with_correct``).  Training on the GPU's sub-pixel path computes the loss
        in the 1x1 head's epilogue (``subpixel.decoder_head_xent``: the logits are never stored);
        otherwise ``softmax_xent(self(x), labels)``."""
        from ..ops import softmax_xent

        if x.dim() == 4:
            x = x.unsqueeze(-1)
        d, h = self.dec, self.head
        if self.training:
            z = x
            for i, c in enumerate(self.enc):
                z = c(z, conv_next=i < len(self.enc) - 1)
            if subpixel.gpu_ok(z, d.cout, z.shape[-1]) and bn_ops.fused_pointwise_ok(z, d.cout, h.cout, d.act) \
                    and subpixel.xent_ok(d.cout, h.cout):
                loss, hits = subpixel.decoder_head_xent(z, d.weight, d.gamma, d.beta, d.running_mean, d.running_var,
                                                        h.weight, h.bias, labels, d.bn_momentum, d.bn_eps, d.act,
                                                        smoothing, want_hits=with_correct)
                return (loss, hits) if with_correct else loss
            return softmax_xent(self._decode(z), labels, smoothing, with_correct)
        return softmax_xent(self(x), labels, smoothing, with_correct)
