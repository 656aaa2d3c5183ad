#!/usr/bin/env python3
"""Cycle stamps of conv_tile's compute wave 0 and loader (FN_TILE_DBG=16, experiments build) for the
FeatureNet-3D step, eager, with the BN prologue on or off (FN_BN_PROLOGUE): where the loader's time
goes -- DMA issue + landing ("job") against the prologue transform ("epilogue" of the loader).

    FN_BUILD_EXPERIMENTS=1 python -c 'import __graft_entry__ as g; g.build()'
    FN_TILE_DBG=16 FN_BN_PROLOGUE=1 python scripts/diag_prologue_stamps.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from featurenet_amd.models.featurenet3d import FeatureNet3D
    from featurenet_amd.ops import softmax_xent
    from featurenet_amd.training.flat import FlatParams

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = FeatureNet3D().to(dev)
    flat = FlatParams(model)
    x = (torch.rand(128, 64, 64, 64, 1, device=dev) < 0.3).to(torch.uint8)
    y = torch.randint(0, 24, (128,), device=dev)
    for it in range(3):
        print(f"--- step {it}", file=sys.stderr, flush=True)
        flat.zero_grad()
        softmax_xent(model(x), y).backward()
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
