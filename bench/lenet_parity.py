#!/usr/bin/env python3
"""The reference's behavioural check: learning curves of the FeatureNet-built ``lenet5`` template
against a hand-written LeNet-5 (``/root/reference/full_lenet5.py:48-54`` writes 10 template runs,
``lenet5.py:84-86`` the hand-written ones, ``plots/plotter.py:128-169`` plots their mean training
and test accuracy per epoch).

Here both run on the framework (``models/baselines.py`` LeNet5 is the hand-written network;
``ir`` compiles the ``lenet5`` template), ``--runs`` seeds each, on the same dataset, and the two
groups go into one report file in the reference's line format; ``utils/analysis.compare_accuracy``
draws the mean curves (SVG).  The reference trains the hand-written model with SGD and the
template with Adam (its ``TensorflowGenerator``); ``--optimizer`` picks one for both (default: as
the reference).  CIFAR-10 is not downloadable here: without files under the data roots the
dataset is the class-conditional synthetic set of ``training/data.py`` (the numbers are then
first-party, "parity unpinned").

    python bench/lenet_parity.py --runs 3 --epochs 12 --out profiles/r6_lenet5_template_vs_handwritten.svg
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def hard_synthetic(ds, sizes, seed: int = 0):
    """The class-blob stand-in made hard enough to separate the two curves: blob amplitude 0.25 on
    N(0.3, 0.3) noise, the blob centre jittered +-3 pixels, radius 2-3."""
    from featurenet_amd.training.data import Dataset

    g = np.random.default_rng(seed)
    H, W, C = ds.input_shape

    def make(n):
        y = g.integers(0, ds.num_classes, n)
        x = g.normal(0.3, 0.3, (n, H, W, C)).astype(np.float32)
        cy = (y * 7 % max(H - 6, 1)) + 3 + g.integers(-3, 4, n)
        cx = (y * 13 % max(W - 6, 1)) + 3 + g.integers(-3, 4, n)
        r2 = g.integers(4, 10, n)
        yy, xx = np.mgrid[0:H, 0:W]
        for i in range(n):
            x[i, (yy - cy[i]) ** 2 + (xx - cx[i]) ** 2 < r2[i], :] += 0.25
        return np.clip(x, 0, 1), y.astype(np.int64)

    xtr, ytr = make(sizes[0])
    xte, yte = make(sizes[1])
    return Dataset(ds.name + "-hard", xtr, ytr, xte, yte, ds.num_classes, ds.input_shape, synthetic=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dataset", default="cifar")
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--epochs", type=int, default=12)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--optimizer", choices=["reference", "adam", "sgd"], default="reference")
    ap.add_argument("--sizes", type=int, nargs=2, default=(12000, 2000), help="synthetic train / test sizes")
    ap.add_argument("--out", default="lenet5_parity.svg")
    ap.add_argument("--report", default=None)
    ap.add_argument("--hard", action="store_true",
                    help="without CIFAR files: a harder synthetic set (faint, jittered class blobs in strong noise) -- "
                         "the default stand-in is separable after one epoch, so both curves sit at 1.0")
    a = ap.parse_args()

    from featurenet_amd.api import build_model
    from featurenet_amd.models.baselines import build_baseline
    from featurenet_amd.training.data import load_dataset
    from featurenet_amd.training.trainer import Trainer
    from featurenet_amd.utils.analysis import compare_accuracy
    from featurenet_amd.utils.reports import report_line

    ds = load_dataset(a.dataset, synthetic_sizes=tuple(a.sizes))
    if a.hard and ds.synthetic:
        ds = hard_synthetic(ds, a.sizes)
    report = a.report or os.path.join(tempfile.mkdtemp(), "report_lenet5_parity.txt")
    lines, summary = [], {"standard": [], "featurenet": []}
    for kind in ("standard", "featurenet"):               # compare_accuracy: first group = standard
        for run in range(a.runs):
            torch.manual_seed(run)
            if kind == "standard":
                model = build_baseline("lenet5-handwritten", ds.input_shape, ds.num_classes)
                opt = "sgd" if a.optimizer == "reference" else a.optimizer
                lr = 0.01 if opt == "sgd" else 1e-3
            else:
                model, _ = build_model("lenet5", ds.input_shape, ds.num_classes)
                opt = "adam" if a.optimizer == "reference" else a.optimizer
                lr = 1e-3 if opt == "adam" else 0.01
            tr = Trainer(model, optimizer=opt, lr=lr, graph=True)
            t0 = time.time()
            hist = tr.fit(ds.x_train, ds.y_train, epochs=a.epochs, batch_size=a.batch,
                          validation_data=(ds.x_test, ds.y_test), callbacks=[], verbose=0, seed=run)
            _, acc = tr.evaluate(ds.x_test, ds.y_test)
            nparams = sum(p.numel() for p in model.parameters())
            lines.append(report_line(len(lines), float(acc), False, time.time() - t0, nparams, 0,
                                     {"acc": list(hist.history["acc"]), "val_acc": list(hist.history["val_acc"])}))
            summary[kind].append(round(float(acc), 4))
            print(f"{kind} run {run}: test acc {acc:.4f} ({opt}, {nparams} params, {time.time() - t0:.1f} s)",
                  flush=True)
    with open(report, "w") as f:
        f.write("".join(lines))
    out = compare_accuracy(report, a.out, group=a.runs, epochs=a.epochs)
    res = {"dataset": ds.name, "synthetic": bool(ds.synthetic), "epochs": a.epochs, "runs": a.runs,
           "test_acc": summary, "mean": {k: round(float(np.mean(v)), 4) for k, v in summary.items()},
           "plot": str(out), "report": report}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
