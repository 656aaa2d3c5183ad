#!/usr/bin/env python3
"""Top-1 accuracy of FeatureNet-3D on the procedural machining-feature set.

The second half of BASELINE.json's metric ("samples/sec ...; top-1 acc"):
train FeatureNet-3D (64^3, 24 classes, bf16 kernels, Adam 1e-3, batch 128)
from random init on the procedural voxel dataset of ``csrc/runtime/voxel.cpp``
(24 machining-feature classes carved into a stock block, random orientation),
then report held-out top-1 accuracy, the training throughput of the whole run
(data loading and bit-unpacking included) and a checkpoint round trip
through ``classify()``.

    python bench/accuracy.py --train-per-class 400 --test-per-class 50 --epochs 6
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench/accuracy.py

The dataset is synthetic (no network for the real FeatureNet CAD set); the
reference repository publishes no accuracy for this task, so the number is
first-party ("parity unpinned").
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--classes", type=int, default=24)
    ap.add_argument("--train-per-class", type=int, default=400)
    ap.add_argument("--test-per-class", type=int, default=50)
    ap.add_argument("--epochs", type=int, default=6)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--fp8", action="store_true",
                    help="also quantise the trained model to fp8 (inference/fp8.py) and report its held-out top-1")
    a = ap.parse_args()

    import featurenet_amd as fn
    from featurenet_amd.parallel.ddp import init_from_env
    from featurenet_amd.training.data import voxel_dataset

    rank, world, local = init_from_env()
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    t0 = time.time()
    ds = voxel_dataset(a.train_per_class * a.classes, a.test_per_class * a.classes, size=a.size,
                       num_classes=a.classes, seed=a.seed)
    t_gen = time.time() - t0
    ckpt = os.path.join(tempfile.mkdtemp(), "fn3d.fnk")
    t0 = time.time()
    res = fn.train("featurenet3d", data=ds, epochs=a.epochs, batch_size=a.batch, lr=a.lr, seed=a.seed,
                   save_path=ckpt if rank == 0 else None, verbose=1 if rank == 0 else 0, callbacks=[])
    t_train = time.time() - t0
    hist = res.history
    out = {
        "metric": "top-1 accuracy (64^3 voxel, 24-class, procedural machining features)",
        "value": round(res.accuracy, 4),
        "unit": "fraction",
        "n_gpus": world,
        "epochs": a.epochs,
        "train_samples": len(ds.y_train),
        "test_samples": len(ds.y_test),
        "train_acc_last_epoch": round(hist["acc"][-1], 4),
        "val_acc_per_epoch": [round(v, 4) for v in hist.get("val_acc", [])],
        "loss_per_epoch": [round(v, 4) for v in hist["loss"]],
        "train_samples_per_s_per_epoch": [round(v, 1) for v in hist["samples_per_s"]],
        "train_wall_s": round(t_train, 2),
        "datagen_s": round(t_gen, 2),
        "dtype": "bf16",
        "data": "synthetic procedural voxels (featurenet_amd._rt.generate_voxels), random-init weights",
        "config": {"model": "FeatureNet-3D", "global_batch": a.batch * world, "optimizer": "adam",
                   "lr": a.lr, "parallelism": f"dp{world}"},
    }
    if rank == 0:
        labels, _ = fn.classify(ckpt, ds.x_test, packed_size=a.size)
        out["classify_roundtrip_acc"] = round(float((labels == np.asarray(ds.y_test)).mean()), 4)
        if a.fp8:
            out["fp8"] = fp8_parity(res.model, ds, a.size)
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


@torch.no_grad()
def fp8_parity(model, ds, size: int, calib: int = 256, chunk: int = 128) -> dict:
    """Post-training fp8 quantisation of the trained model (activation scales calibrated on
    ``calib`` training samples), then held-out top-1 of fp8 vs bf16 and their agreement."""
    from featurenet_amd.inference.fp8 import quantize_model
    from featurenet_amd.training.data import unpack_voxels

    dev = next(model.parameters()).device
    model.eval()

    def batch(xs, i, n):
        xb = torch.as_tensor(np.asarray(xs[i:i + n])).to(dev)
        return unpack_voxels(xb, size).to(torch.bfloat16)

    cx = batch(ds.x_train, 0, calib)
    q = quantize_model(model, cx)                          # the default stem (FN_F8_STEM)
    qs = quantize_model(model, cx, fp8_stem=False)         # bf16 stem writing e4m3 from its epilogue
    from featurenet_amd.ops.conv_tile import experiments_built

    # int8 stem (v_mfma_i32_16x16x64_i8): an experiment build only (FN_BUILD_EXPERIMENTS=1)
    qi = quantize_model(model, cx, fp8_stem="i8") if experiments_built() else None
    y = np.asarray(ds.y_test)
    pb, pq, ps, pi, pt = [], [], [], [], []
    for i in range(0, len(y), chunk):
        xb = batch(ds.x_test, i, chunk)
        pb.append(model(xb).float().argmax(-1).cpu())
        pq.append(q(xb).float().argmax(-1).cpu())
        ps.append(qs(xb).float().argmax(-1).cpu())
        if qi is not None:
            pi.append(qi(xb).float().argmax(-1).cpu())
        os.environ["FN_F8_BLOCK"] = "0"                 # the per-tensor activation scales, same model
        try:
            pt.append(qs(xb).float().argmax(-1).cpu())
        finally:
            os.environ.pop("FN_F8_BLOCK")
    pb, pq, ps, pt = (torch.cat(t).numpy() for t in (pb, pq, ps, pt))
    acc_b, acc_q, acc_s, acc_t = (float((t == y).mean()) for t in (pb, pq, ps, pt))
    i8 = None
    if qi is not None:
        pi = torch.cat(pi).numpy()
        acc_i = float((pi == y).mean())
        i8 = {"top1_fp8": round(acc_i, 4), "drop_pt": round(100 * (acc_b - acc_i), 2),
              "agreement": round(float((pb == pi).mean()), 4)}
    return {"top1_bf16": round(acc_b, 4), "top1_fp8": round(acc_q, 4), "drop_pt": round(100 * (acc_b - acc_q), 2),
            "agreement": round(float((pb == pq).mean()), 4), "calib_samples": calib,
            "stem": q.stem and ("i8" if q.stem.int8 else "e4m3") or "bf16",
            "activations": "block-scaled (E8M0 per position x 32 channels)" if q.block_mode(
                (1, size, size, size, 1)) else "per-tensor",
            "bf16_stem": {"top1_fp8": round(acc_s, 4), "drop_pt": round(100 * (acc_b - acc_s), 2),
                          "agreement": round(float((pb == ps).mean()), 4)},
            "per_tensor": {"top1_fp8": round(acc_t, 4), "drop_pt": round(100 * (acc_b - acc_t), 2),
                           "agreement": round(float((pb == pt).mean()), 4)},
            "calib_agreement": q.calib_agreement,
            "i8_stem": i8,
            "kernel": ("conv_halo_f8" if os.environ.get("FN_F8_TILE", "1") == "0" else "conv_tile F8 variant")
                      + " (v_mfma_scale_f32_16x16x128_f8f6f4, e4m3)"}


if __name__ == "__main__":
    main()
