#!/usr/bin/env python3
"""Per-kernel microbenchmark of FeatureNet-3D's convolutions (batch 128, 64^3).

Times the native forward / dgrad / wgrad kernels of each layer with HIP events
(median of ``--reps`` after warmup) and reports useful TFLOP/s (FLOPs of the
convolution itself, not of padded work).  Used to A/B kernel variants.

    python bench/conv_kernels.py [--batch 128] [--reps 20] [--layers 1,2,3,4]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

LAYERS = {  # name: (input spatial, Cin, Cout, kernel, stride)
    1: (64, 1, 32, 7, 2),
    2: (29, 32, 32, 5, 1),
    3: (25, 32, 64, 4, 1),
    4: (22, 64, 64, 3, 1),
}


def timeit(fn, reps: int, warmup: int = 3, inner: int = 5) -> float:
    """Median over ``reps`` of the mean time of ``inner`` back-to-back calls (ms).

    Back-to-back calls keep the GPU queue full, so host-side launch work of an op
    overlaps its predecessor's kernels instead of being timed as idle GPU time
    (rocprofv3 remains the reference for per-kernel numbers)."""
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(inner):
            fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) / inner)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--layers", default="1,2,3,4")
    a = ap.parse_args()
    import importlib

    C = importlib.import_module("featurenet_amd.ops.conv")
    from featurenet_amd.ops.spec import ConvSpec

    torch.manual_seed(0)
    dev = "cuda"
    total = 0.0
    res = []
    for li in [int(v) for v in a.layers.split(",")]:
        S, ci, co, k, s = LAYERS[li]
        if li == 1:
            x = (torch.rand(a.batch, S, S, S, ci, device=dev) < 0.3).to(torch.bfloat16)
        else:
            x = torch.randn(a.batch, S, S, S, ci, device=dev).to(torch.bfloat16)
        spec = ConvSpec.make(x.shape, co, k, s)
        w = torch.randn(co, k, k, k, ci, device=dev) * 0.05
        dy = torch.randn(spec.out_shape5, device=dev).to(torch.bfloat16)
        flops = 2.0 * spec.M * spec.K * spec.kdim
        xr = x.requires_grad_(li > 1)

        def fwd():
            return C.ConvFn.apply(xr, w, None, spec, 0, True)

        y, _ = fwd()
        ops = {"fwd": fwd}
        if li > 1:
            ops["dgrad"] = lambda: C.native_conv_dgrad(dy, w, spec)
        s2d = C.s2d_plan(spec)
        if s2d is not None:
            f, spec2 = s2d
            x2 = C.s2d_input(x, f, spec2)
            ops["s2d_prep"] = lambda: C.s2d_input(x, f, spec2)
            ops["wgrad"] = lambda: C.native_conv_wgrad(dy, x2, spec2)
        else:
            ops["wgrad"] = lambda: C.native_conv_wgrad(dy, x, spec)
        with torch.no_grad():
            for name, fn in ops.items():
                ms = timeit(fn, a.reps)
                total += ms
                tf = flops / (ms * 1e-3) / 1e12 if name != "s2d_prep" else 0.0
                res.append({"layer": li, "op": name, "ms": round(ms, 4), "tflops": round(tf, 1)})
                print(f"conv{li} {name:8s} {ms * 1e3:8.1f} us  {tf:7.1f} TFLOP/s", flush=True)
    print(json.dumps({"total_ms": round(total, 4), "kernels": res}))


if __name__ == "__main__":
    main()
