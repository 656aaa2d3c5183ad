"""Diagnose train/eval BatchNorm gaps: eval accuracy with running stats vs batch stats vs recalibrated stats."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import featurenet_amd as fn  # noqa: E402
from featurenet_amd.training.data import DeviceLoader, voxel_dataset  # noqa: E402


def acc(model, ds, train_mode):
    model.train(train_mode)
    loader = DeviceLoader(ds.x_test, ds.y_test, 128, "cuda", shuffle=False, packed_size=64)
    c = n = 0
    with torch.no_grad():
        for xb, yb in loader:
            p = model(xb.to(torch.bfloat16)).argmax(-1)
            c += int((p == yb).sum())
            n += len(yb)
    return c / n


def main():
    ds = voxel_dataset(24 * 300, 24 * 50, size=64, num_classes=24, seed=0)
    res = fn.train("featurenet3d", data=ds, epochs=int(os.environ.get("EPOCHS", "4")), callbacks=[], verbose=1)
    m = res.model
    bns = [c for c in m.convs]
    saved = [(c.running_mean.clone(), c.running_var.clone()) for c in bns]
    print("eval (running stats):", acc(m, ds, False))
    print("train-mode BN (batch stats):", acc(m, ds, True))
    for c, (rm, rv) in zip(bns, saved):
        c.running_mean.copy_(rm)
        c.running_var.copy_(rv)
    for i, c in enumerate(bns):
        print(i, "rm", c.running_mean[:4].tolist(), "rv", c.running_var[:4].tolist())
    # recalibrate: cumulative average over training batches
    for c in bns:
        c.running_mean.zero_()
        c.running_var.fill_(1)
        c.bn_momentum_saved = c.bn_momentum
    m.train()
    loader = DeviceLoader(ds.x_train, ds.y_train, 128, "cuda", shuffle=True, packed_size=64)
    with torch.no_grad():
        for k, (xb, yb) in enumerate(loader):
            for c in bns:
                c.bn_momentum = 1.0 / (k + 1)
            m(xb.to(torch.bfloat16))
            if k >= 40:
                break
    for i, c in enumerate(bns):
        print(i, "recal rm", c.running_mean[:4].tolist(), "rv", c.running_var[:4].tolist())
    print("eval (recalibrated):", acc(m, ds, False))


if __name__ == "__main__":
    main()
