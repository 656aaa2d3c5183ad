#!/usr/bin/env python3
"""FeatureNet-3D FC1 on the native dense kernels (dense.hip) at the training batch: forward with
several split-K slice counts, dgrad and weight gradient, us per call (events around R launches,
after one warm call).  One JSON line.

    python scripts/bench_fc_native.py --batch 128 --reps 50
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from featurenet_amd import _native  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--features", type=int, default=64000)
    ap.add_argument("--hidden", type=int, default=128)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    M, K, N = a.batch, a.features, a.hidden
    Kn = _native.kernels()
    st = _native.stream(None)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, K, device="cuda") * 0.01
    b = torch.zeros(N, device="cuda")
    g = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    res = {"S_default": int(Kn.dense_splits(M, N, K))}
    for S in sorted({32, 64, 125, 250, 500, 1000, res["S_default"]}):
        part = torch.empty(S, M, N, device="cuda")
        res[f"fwd_S{S}"] = timeit(lambda: Kn.dense_fwd(x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(),
                                                        part.data_ptr(), M, N, K, S, 1, 0, st), a.reps)
    dx = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
    res["dgrad"] = timeit(lambda: Kn.dense_dgrad(g.data_ptr(), w.data_ptr(), dx.data_ptr(), M, N, K, st), a.reps)
    dw = torch.zeros(N, K, device="cuda")
    db = torch.zeros(N, device="cuda")
    S = int(Kn.dense_wgrad_slices(M, N, K))
    part = torch.empty(max(1, S * (N * K + N)), device="cuda")
    res["wgrad_S"] = S
    res["wgrad"] = timeit(lambda: Kn.dense_wgrad(g.data_ptr(), x.data_ptr(), dw.data_ptr(), db.data_ptr(), M, N, K,
                                                 st, [], part.data_ptr(), S, 0, 0), a.reps)
    gb = (x.numel() * 2 + w.numel() * 4) / 1e9
    res["fwd_bytes_gb"] = round(gb, 4)
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
