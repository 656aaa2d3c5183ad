#!/usr/bin/env python3
"""FP8 vs bf16 inference throughput of FeatureNet-3D (BASELINE config 5).

    python bench/infer_fp8.py --size 128 --batch 1024 --chunk 128

Random-init weights (BN running stats at their init values), synthetic binary
voxels.  Prints one JSON line per precision: samples/s over ``--steps`` full
batches (processed ``--chunk`` samples per forward), plus the top-1 agreement
of fp8 with bf16 on the first chunk.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--chunk", type=int, default=128)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--only", choices=["bf16", "fp8"], default=None, help="time one precision (profiling)")
    ap.add_argument("--voxels", choices=["uint8", "bf16"], default="uint8", help="input voxel storage")
    a = ap.parse_args()
    from featurenet_amd.inference.fp8 import quantize_model
    from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig

    torch.manual_seed(0)
    dev = torch.device("cuda")
    m = FeatureNet3D(FeatureNet3DConfig(input_size=a.size, num_classes=24)).to(dev).eval()
    # binary voxels as uint8 (the space-to-depth stem packing reads the bytes); calibration in bf16
    x = (torch.rand(a.chunk, a.size, a.size, a.size, 1, device=dev) < 0.3).to({"uint8": torch.uint8, "bf16": torch.bfloat16}[a.voxels])
    q = quantize_model(m, x[: min(32, a.chunk)].to(torch.bfloat16))
    nchunks = max(1, a.batch // a.chunk)
    res = {}
    with torch.no_grad():
        agree = (m(x).argmax(-1) == q(x).argmax(-1)).float().mean().item()
        for name, fn in (("bf16", m), ("fp8", q)):
            if a.only and name != a.only:
                continue
            for _ in range(a.warmup):
                for _ in range(nchunks):
                    fn(x)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                for _ in range(nchunks):
                    fn(x)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            res[name] = a.steps * nchunks * a.chunk / dt
            print(json.dumps({"metric": f"samples/sec ({a.size}^3 voxel) inference", "precision": name,
                              "value": round(res[name], 1), "unit": "samples/s", "batch": a.batch,
                              "chunk": a.chunk, "ms_per_batch": round(dt / a.steps * 1e3, 2)}), flush=True)
    if len(res) == 2:
        print(json.dumps({"fp8_speedup": round(res["fp8"] / res["bf16"], 3), "top1_agreement_fp8_vs_bf16": agree}))


if __name__ == "__main__":
    main()
