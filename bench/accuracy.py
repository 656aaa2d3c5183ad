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
    python bench/accuracy.py --impl torch --torch-dtype fp32     # the stock-PyTorch fp32 oracle

``--impl torch`` trains the SAME network in stock PyTorch (``nn.functional.conv3d`` /
``batch_norm`` / ``max_pool3d`` / ``linear``, MIOpen + hipBLASLt) from the SAME initial weights
(the native model built with the same seed, its tensors copied over), on the same batches in the
same order (``DeviceLoader``: the shuffle is a function of (seed, epoch)), with the same Keras-style
Adam and the same PreciseBN recalibration -- fp32 throughout (``--torch-dtype fp32``) or bf16
autocast.  It is the convergence oracle for the native bf16 kernels: the reference's only
behavioural check is a learning-curve comparison (``/root/reference/full_lenet5.py:48-54``,
``plots/plotter.py:128-169``), and its own Keras numerics cannot run here.

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
    ap.add_argument("--impl", choices=["native", "torch"], default="native",
                    help="native: the framework's bf16 HIP kernels; torch: the stock-PyTorch oracle (see above)")
    ap.add_argument("--torch-dtype", choices=["fp32", "bf16"], default="fp32",
                    help="--impl torch: fp32 throughout, or bf16 autocast (fp32 master weights)")
    ap.add_argument("--weights-hash", action="store_true",
                    help="also print a sha256 of the trained weights (bitwise run-to-run / box-to-box checks)")
    a = ap.parse_args()
    if a.impl == "torch":
        return torch_oracle(a)

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
    if a.weights_hash:
        out["weights_sha256"] = weights_hash(res.model)
    if rank == 0:
        labels, _ = fn.classify(ckpt, ds.x_test, packed_size=a.size)
        out["classify_roundtrip_acc"] = round(float((labels == np.asarray(ds.y_test)).mean()), 4)
        if a.fp8:
            out["fp8"] = fp8_parity(res.model, ds, a.size)
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def weights_hash(model) -> str:
    """sha256 over every parameter and buffer (name order), as raw bytes."""
    import hashlib

    h = hashlib.sha256()
    for name, t in sorted(list(model.state_dict().items())):
        h.update(name.encode())
        h.update(t.detach().cpu().contiguous().view(torch.uint8).numpy().tobytes() if t.numel() else b"")
    return h.hexdigest()[:16]


class OracleFeatureNet3D(torch.nn.Module):
    """FeatureNet-3D in stock PyTorch ops with the native model's parameters (layouts converted:
    conv weight [K, KD, KH, KW, C] -> [K, C, KD, KH, KW]; the flatten before FC1 is channels-last,
    as the native model's)."""

    def __init__(self, native):
        super().__init__()
        nn = torch.nn
        self.strides, self.bn = [], []
        self.w = nn.ParameterList()
        self.gamma, self.beta = nn.ParameterList(), nn.ParameterList()
        for i, c in enumerate(native.convs):
            self.w.append(nn.Parameter(c.weight.detach().float().permute(0, 4, 1, 2, 3).contiguous().clone()))
            self.gamma.append(nn.Parameter(c.gamma.detach().float().clone()))
            self.beta.append(nn.Parameter(c.beta.detach().float().clone()))
            self.register_buffer(f"rm{i}", c.running_mean.detach().float().clone())
            self.register_buffer(f"rv{i}", c.running_var.detach().float().clone())
            self.strides.append(c.stride if isinstance(c.stride, int) else c.stride[0])
            self.bn.append((c.bn_momentum, c.bn_eps))
        self.pool = native.convs[-1].pool[0] if native.convs[-1].pool else 1
        self.fc1_w = nn.Parameter(native.fc1.weight.detach().float().clone())
        self.fc1_b = nn.Parameter(native.fc1.bias.detach().float().clone())
        self.fc2_w = nn.Parameter(native.fc2.weight.detach().float().clone())
        self.fc2_b = nn.Parameter(native.fc2.bias.detach().float().clone())
        self.bn_momentum_override = None

    def forward(self, x):                              # x: [N, S, S, S, 1]
        F = torch.nn.functional
        h = x.permute(0, 4, 1, 2, 3)
        if h.is_cuda:
            h = h.contiguous(memory_format=torch.channels_last_3d)
        for i in range(len(self.w)):
            h = F.conv3d(h, self.w[i].to(h.dtype) if h.dtype != torch.float32 else self.w[i], stride=self.strides[i])
            mom, eps = self.bn[i]
            if self.bn_momentum_override is not None:
                mom = self.bn_momentum_override
            h = F.batch_norm(h, getattr(self, f"rm{i}"), getattr(self, f"rv{i}"), self.gamma[i], self.beta[i],
                             self.training, mom, eps)
            h = F.relu(h)
        if self.pool > 1:
            h = F.max_pool3d(h, self.pool)
        f = h.permute(0, 2, 3, 4, 1).flatten(1)
        return F.linear(F.relu(F.linear(f, self.fc1_w, self.fc1_b)), self.fc2_w, self.fc2_b)


def torch_oracle(a) -> None:
    """Train the stock-PyTorch FeatureNet-3D (fp32 or bf16 autocast) from the native model's
    initial weights on the same batch sequence; print the same JSON fields as the native run."""
    import math

    from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig
    from featurenet_amd.training.data import DeviceLoader, voxel_dataset

    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    # MIOpen find mode (time the solvers once per shape, keep the fastest) and channels-last 3-D
    # tensors: without them stock PyTorch runs MIOpen's fallback 3-D kernels (~100 samples/s,
    # bench.py --impl torch); the math is the same
    torch.backends.cudnn.benchmark = True
    t0 = time.time()
    # (MIOpen's first find of each 3-D fp32 shape compiles and times its solvers for minutes without
    # printing anything: a heartbeat keeps a supervised run visibly alive)
    import threading

    def beat():
        while True:
            time.sleep(30)
            print(f"  [{time.time() - t0:.0f} s]", flush=True)

    threading.Thread(target=beat, daemon=True).start()
    ds = voxel_dataset(a.train_per_class * a.classes, a.test_per_class * a.classes, size=a.size,
                       num_classes=a.classes, seed=a.seed)
    t_gen = time.time() - t0
    torch.manual_seed(a.seed)                           # the native api.train's initial weights
    native = FeatureNet3D(FeatureNet3DConfig(input_size=a.size, num_classes=a.classes))
    model = OracleFeatureNet3D(native).to(dev)
    if dev.type == "cuda":
        for w in model.w:
            w.data = w.data.contiguous(memory_format=torch.channels_last_3d)
    params = [p for p in model.parameters()]
    m = [torch.zeros_like(p) for p in params]
    v = [torch.zeros_like(p) for p in params]
    b1, b2, eps, lr = 0.9, 0.999, 1e-7, a.lr            # FlatAdam defaults (Keras-2.2 epsilon placement)
    amp = a.torch_dtype == "bf16" and dev.type == "cuda"
    loader = DeviceLoader(ds.x_train, ds.y_train, a.batch, dev, shuffle=True, packed_size=a.size, seed=a.seed,
                          even=True, dtype=torch.float32)
    val = DeviceLoader(ds.x_test, ds.y_test, a.batch, dev, shuffle=False, packed_size=a.size, even=False,
                       dtype=torch.float32)
    t_step = 0

    def prep(xb):
        return xb.float()

    @torch.no_grad()
    def evaluate():
        model.eval()
        hit, n, ls = 0, 0, 0.0
        for xb, yb in val:
            with torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=amp):
                lg = model(prep(xb)).float()
            ls += float(torch.nn.functional.cross_entropy(lg, yb, reduction="sum"))
            hit += int((lg.argmax(-1) == yb).sum())
            n += yb.numel()
        return ls / max(n, 1), hit / max(n, 1)

    @torch.no_grad()
    def precise_bn(epoch, batches=32):                  # Trainer.recalibrate_bn: running stats = mean over
        model.train()                                    # 32 shuffled batches (momentum 1/(k+1))
        d = loader.derived(seed=a.seed + epoch + 7919)
        for k, (xb, _) in enumerate(d):
            if k >= batches:
                break
            model.bn_momentum_override = 1.0 / (k + 1)
            with torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=amp):
                model(prep(xb))
        model.bn_momentum_override = None

    hist = {"loss": [], "acc": [], "val_acc": [], "val_loss": [], "samples_per_s": []}
    t_train0 = time.time()
    for epoch in range(a.epochs):
        model.train()
        loader.set_epoch(epoch)
        te = time.time()
        lsum, hits, seen = 0.0, 0, 0
        for bi, (xb, yb) in enumerate(loader):
            with torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=amp):
                lg = model(prep(xb)).float()
            loss = torch.nn.functional.cross_entropy(lg, yb)
            if bi % 40 == 0:                             # (progress: a long epoch stays visibly alive)
                print(f"  epoch {epoch + 1} batch {bi}", flush=True)
            for p in params:
                p.grad = None
            loss.backward()
            t_step += 1
            bc1, bc2 = 1.0 - b1 ** t_step, 1.0 - b2 ** t_step
            lr_t = lr * math.sqrt(bc2) / bc1
            with torch.no_grad():
                for p, mm, vv in zip(params, m, v):
                    mm.mul_(b1).add_(p.grad, alpha=1 - b1)
                    vv.mul_(b2).addcmul_(p.grad, p.grad, value=1 - b2)
                    p.addcdiv_(mm, vv.sqrt().add_(eps), value=-lr_t)
            lsum += float(loss) * yb.numel()
            hits += int((lg.argmax(-1) == yb).sum())
            seen += yb.numel()
        hist["loss"].append(lsum / seen)
        hist["acc"].append(hits / seen)
        hist["samples_per_s"].append(seen / max(time.time() - te, 1e-9))
        precise_bn(epoch)
        vl, va = evaluate()
        hist["val_loss"].append(vl)
        hist["val_acc"].append(va)
        print(f"epoch {epoch + 1}/{a.epochs} loss={hist['loss'][-1]:.4g} acc={hist['acc'][-1]:.4g} "
              f"val_acc={va:.4g}", flush=True)
    out = {
        "metric": "top-1 accuracy (64^3 voxel, 24-class, procedural machining features)",
        "value": round(hist["val_acc"][-1], 4),
        "unit": "fraction",
        "impl": f"torch-{a.torch_dtype}",
        "n_gpus": 1,
        "epochs": a.epochs,
        "seed": a.seed,
        "train_samples": len(ds.y_train),
        "test_samples": len(ds.y_test),
        "train_acc_last_epoch": round(hist["acc"][-1], 4),
        "val_acc_per_epoch": [round(x, 4) for x in hist["val_acc"]],
        "loss_per_epoch": [round(x, 4) for x in hist["loss"]],
        "train_samples_per_s_per_epoch": [round(x, 1) for x in hist["samples_per_s"]],
        "train_wall_s": round(time.time() - t_train0, 2),
        "datagen_s": round(t_gen, 2),
        "dtype": "fp32" if not amp else "bf16 autocast",
        "data": "synthetic procedural voxels (featurenet_amd._rt.generate_voxels), random-init weights",
        "config": {"model": "FeatureNet-3D (stock PyTorch ops, same init as the native run)",
                   "global_batch": a.batch, "optimizer": "adam (Keras-2.2 epsilon)", "lr": a.lr},
    }
    print(json.dumps(out), flush=True)


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
    # the calibration check deciding the numerics (block scales -> per-tensor -> bf16)
    qa = quantize_model(model, cx, fallback=True)
    y = np.asarray(ds.y_test)
    pb, pq, ps, pi, pt, pa = [], [], [], [], [], []
    for i in range(0, len(y), chunk):
        xb = batch(ds.x_test, i, chunk)
        pb.append(model(xb).float().argmax(-1).cpu())
        pq.append(q(xb).float().argmax(-1).cpu())
        ps.append(qs(xb).float().argmax(-1).cpu())
        if qi is not None:
            pi.append(qi(xb).float().argmax(-1).cpu())
        pa.append(qa(xb).float().argmax(-1).cpu())
        os.environ["FN_F8_BLOCK"] = "0"                 # the per-tensor activation scales, same model
        try:
            pt.append(qs(xb).float().argmax(-1).cpu())
        finally:
            os.environ.pop("FN_F8_BLOCK")
    pb, pq, ps, pt, pa = (torch.cat(t).numpy() for t in (pb, pq, ps, pt, pa))
    acc_b, acc_q, acc_s, acc_t, acc_a = (float((t == y).mean()) for t in (pb, pq, ps, pt, pa))
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
            "auto_fallback": {"mode": qa.calib_history[-1][0], "calib_history": qa.calib_history,
                              "top1_fp8": round(acc_a, 4), "drop_pt": round(100 * (acc_b - acc_a), 2),
                              "agreement": round(float((pb == pa).mean()), 4)},
            "i8_stem": i8,
            "kernel": ("conv_halo_f8" if os.environ.get("FN_F8_TILE", "1") == "0" else "conv_tile F8 variant")
                      + " (v_mfma_scale_f32_16x16x128_f8f6f4, e4m3)"}


if __name__ == "__main__":
    main()
