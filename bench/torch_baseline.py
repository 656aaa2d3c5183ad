"""First-party comparison baseline: stock PyTorch-ROCm eager FeatureNet-3D.

The reference publishes no throughput numbers, so the number
``bench.py`` is compared against is this: the same FeatureNet-3D
architecture, the same synthetic 64^3 data, batch and bf16 setting, built
from stock ``nn.Conv3d`` / ``nn.BatchNorm3d`` / ``nn.MaxPool3d`` (MIOpen),
``nn.Linear`` (hipBLASLt), ``torch.optim.Adam`` and
``DistributedDataParallel`` over RCCL.  Run it through ``bench.py --impl torch``.
"""
from __future__ import annotations

import torch
from torch import nn


class TorchFeatureNet3D(nn.Module):
    def __init__(self, input_size=64, in_channels=1, num_classes=24, widths=(32, 32, 64, 64), kernels=(7, 5, 4, 3),
                 strides=(2, 1, 1, 1), pool=2, fc=128):
        super().__init__()
        layers = []
        cin = in_channels
        s = input_size
        for w, k, st in zip(widths, kernels, strides):
            layers += [nn.Conv3d(cin, w, k, st, bias=False), nn.BatchNorm3d(w), nn.ReLU(inplace=True)]
            cin = w
            s = (s - k) // st + 1
        layers.append(nn.MaxPool3d(pool))
        s //= pool
        self.features = nn.Sequential(*layers)
        self.fc1 = nn.Linear(s ** 3 * cin, fc)
        self.fc2 = nn.Linear(fc, num_classes)

    def forward(self, x):  # x: [N, 1, S, S, S]
        f = self.features(x).flatten(1)
        return self.fc2(torch.relu(self.fc1(f)))
