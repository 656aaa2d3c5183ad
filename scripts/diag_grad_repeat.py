#!/usr/bin/env python3
"""Two identical backward passes of the DDP-test FeatureNet-3D config in one process:
per-parameter relative difference of the flat gradients (kernel determinism check)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig  # noqa: E402
from featurenet_amd.ops import softmax_xent  # noqa: E402
from featurenet_amd.training.flat import FlatParams  # noqa: E402

CFG = dict(input_size=16, num_classes=4, widths=(16, 16, 32, 32), kernels=(3, 3, 3, 3), strides=(1, 1, 1, 1), fc=32)
dev = torch.device("cuda", 0)
torch.manual_seed(100)
model = FeatureNet3D(FeatureNet3DConfig(**CFG)).to(dev)
flat = FlatParams(model)
g = torch.Generator().manual_seed(3)
x = (torch.rand(8, 16, 16, 16, 1, generator=g) < 0.3).to(torch.bfloat16).to(dev)
y = torch.randint(0, 4, (8,), generator=g).to(dev)
grads = []
for _ in range(3):
    flat.zero_grad()
    softmax_xent(model(x), y).backward()
    torch.cuda.synchronize()
    grads.append({n: p.grad.detach().clone() for n, p in model.named_parameters()})
for n in grads[0]:
    a, b, c = grads[0][n], grads[1][n], grads[2][n]
    d1 = ((a - b).norm() / (a.norm() + 1e-30)).item()
    d2 = ((b - c).norm() / (b.norm() + 1e-30)).item()
    if d1 or d2:
        print(f"{n:40s} {tuple(a.shape)} rel(1,2)={d1:.3e} rel(2,3)={d2:.3e}")
print("done")
