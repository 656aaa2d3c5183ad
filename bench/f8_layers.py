#!/usr/bin/env python3
"""Per-layer timing of the 128^3 inference convolutions: fp8 tile kernel vs bf16 tile kernel.

    python bench/f8_layers.py [--batch 128] [--reps 10]

Prints one JSON line per layer with both kernels' times and the achieved fraction of the
dense MFMA peak (bf16 2.5 PF, fp8 5.0 PF).  ``FN_F8_DBG`` (1 / 2 / 4) runs the fp8 kernel's
timing-only experiment variants (no weight loads / no halo reads / no halo DMA).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

LAYERS = {2: (61, 32, 32, 5), 3: (57, 32, 64, 4), 4: (54, 64, 64, 3)}   # 128^3 input after the stride-2 stem


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--layers", default="2,3,4")
    ap.add_argument("--no-bf16", action="store_true")
    a = ap.parse_args()
    from bench.conv_kernels import timeit
    from featurenet_amd import ops
    from featurenet_amd.inference.fp8 import Fp8Conv, quantize_fp8_act
    from featurenet_amd.models.layers import Conv
    from featurenet_amd.ops.spec import ConvSpec

    torch.manual_seed(0)
    dev = "cuda"
    for li in [int(v) for v in a.layers.split(",")]:
        S, ci, co, k = LAYERS[li]
        conv = Conv(ci, co, (k, k, k), 1, "valid", bn=False, act="relu").to(dev).eval()
        x = torch.relu(torch.randn(a.batch, S, S, S, ci, device=dev)).to(torch.bfloat16)
        spec = ConvSpec.make(tuple(x.shape), co, k, 1)
        flops = 2.0 * spec.M * spec.K * spec.kdim
        f8 = Fp8Conv(conv, float(x.float().amax()) / 448.0, None, relu=True)
        xq = quantize_fp8_act(x, float(x.float().amax()) / 448.0)
        t8 = timeit(lambda: f8(xq, tuple(x.shape)), a.reps, inner=2)
        r = {"layer": f"conv{li}", "batch": a.batch, "dbg": int(os.environ.get("FN_F8_DBG", "0")),
             "fp8_ms": round(t8, 3), "fp8_pct_peak": round(100 * flops / (t8 * 1e-3) / 5.0e15, 1)}
        if not a.no_bf16:
            w = conv.weight.detach().float()
            tb = timeit(lambda: ops.conv(x, w, None, spec, "relu"), a.reps, inner=2)
            r.update(bf16_ms=round(tb, 3), bf16_pct_peak=round(100 * flops / (tb * 1e-3) / 2.5e15, 1),
                     speedup=round(tb / t8, 3))
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
