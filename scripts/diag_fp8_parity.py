#!/usr/bin/env python3
"""Where an fp8 model's disagreement with its bf16 model comes from: train FeatureNet-3D as
``bench/accuracy.py`` does (deterministic training: the same seed gives the same model), then run
the held-out set through the bf16 model, the block-scaled fp8 path and the per-tensor fp8 path,
keeping every conv layer's output, and report per layer the relative L2 error of each fp8 path
against the bf16 activations (dequantised), the share of saturated / flushed-to-zero values, and
the top-1 agreement.  One JSON line per layer, then a summary.

    python scripts/diag_fp8_parity.py --seed 3 --epochs 16 --train-per-class 1000
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--epochs", type=int, default=16)
    ap.add_argument("--train-per-class", type=int, default=1000)
    ap.add_argument("--test-per-class", type=int, default=50)
    ap.add_argument("--chunk", type=int, default=200)
    a = ap.parse_args()
    import featurenet_amd as fn
    from featurenet_amd import ops
    from featurenet_amd.inference import fp8 as F8
    from featurenet_amd.ops.spec import ConvSpec
    from featurenet_amd.training.data import unpack_voxels, voxel_dataset

    ds = voxel_dataset(a.train_per_class * 24, a.test_per_class * 24, size=64, num_classes=24, seed=a.seed)
    res = fn.train("featurenet3d", data=ds, epochs=a.epochs, batch_size=128, lr=1e-3, seed=a.seed, verbose=0,
                   callbacks=[])
    model = res.model.eval()
    dev = next(model.parameters()).device

    def batch(xs, i, n):
        return unpack_voxels(torch.as_tensor(np.asarray(xs[i:i + n])).to(dev), 64).to(torch.bfloat16)

    q = F8.quantize_model(model, batch(ds.x_train, 0, 256), fp8_stem=False)
    y = np.asarray(ds.y_test)
    nl = len(q.layers) + 1
    err = {k: np.zeros(nl) for k in ("blk", "ten")}
    ref2 = np.zeros(nl)
    sat = {k: np.zeros(nl) for k in ("blk", "ten")}
    pb, pk, pt = [], [], []
    with torch.no_grad():
        for i in range(0, len(y), a.chunk):
            x = batch(ds.x_test, i, a.chunk)
            if x.dim() == 4:
                x = x.unsqueeze(-1)
            # bf16 reference activations (eval convs: BN folded, ReLU, the last with its pool)
            refs, h = [], x
            for c in model.convs:
                h = c(h)
                refs.append(h.float())
            pb.append(model(x).float().argmax(-1).cpu())
            c1 = model.convs[0]
            spec = ConvSpec.make(tuple(x.shape), c1.cout, c1.kernel, c1.stride, c1.padding)
            # block-scaled path
            xq = q._bf16_stem_fp8_out(x, spec, block=True)
            acts = [F8.dequantize_fp8_block(*xq)]
            shape = spec.out_shape5
            for li, layer in enumerate(q.layers):
                last = li == len(q.layers) - 1
                fused = last and q._pool_fusable() and layer.pool_plan(shape, block=True) is not None
                xq, shape = layer(xq, shape, pool=fused)
                acts.append(xq.float() if not isinstance(xq, tuple) else F8.dequantize_fp8_block(*xq))
            blk = acts
            pk.append(q._dense(xq.reshape(xq.shape[0], -1)).float().argmax(-1).cpu())
            # per-tensor path
            os.environ["FN_F8_BLOCK"] = "0"
            try:
                yq = ops.conv(x, q.c1_w, q.c1_b, spec, "relu")
                xt = F8.quantize_fp8_act(yq, q.act_scales[0])
                acts = [xt.view(torch.float8_e4m3fn).float() * q.act_scales[0]]
                shape = spec.out_shape5
                for li, layer in enumerate(q.layers):
                    last = li == len(q.layers) - 1
                    fused = last and q._pool_fusable() and layer.pool_plan(shape) is not None
                    xt, shape = layer(xt, shape, pool=fused)
                    acts.append(xt.float() if xt.dtype != torch.uint8
                                else xt.view(torch.float8_e4m3fn).float() * q.act_scales[li + 1])
                ten = acts
                pt.append(q(x).float().argmax(-1).cpu())
            finally:
                os.environ.pop("FN_F8_BLOCK")
            for li in range(nl):
                r = refs[li]
                ref2[li] += float((r * r).sum())
                for k, v in (("blk", blk[li]), ("ten", ten[li])):
                    v = v.reshape(r.shape)
                    err[k][li] += float(((v - r) ** 2).sum())
                    sat[k][li] += float(((v == 0) & (r > 0)).sum())
    pb, pk, pt = (torch.cat(t).numpy() for t in (pb, pk, pt))
    for li in range(nl):
        print(json.dumps({"layer": li, "rel_l2_block": round(float(np.sqrt(err["blk"][li] / ref2[li])), 5),
                          "rel_l2_tensor": round(float(np.sqrt(err["ten"][li] / ref2[li])), 5),
                          "flushed_block": int(sat["blk"][li]), "flushed_tensor": int(sat["ten"][li])}))
    print(json.dumps({"seed": a.seed, "top1_bf16": float((pb == y).mean()), "top1_block": float((pk == y).mean()),
                      "top1_tensor": float((pt == y).mean()), "agree_block": float((pb == pk).mean()),
                      "agree_tensor": float((pb == pt).mean()), "act_scales": [float(s) for s in q.act_scales]}))


if __name__ == "__main__":
    main()
