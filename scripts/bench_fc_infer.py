#!/usr/bin/env python3
"""FeatureNet-3D FC1 at 128^3 inference (batch chunk 1024, 26^3 x 64 = 1,124,864 features -> 128,
bf16 weight copy) on the native dense forward: the whole chunk in one call at several split-K
slice counts, and the chunk as 8 row blocks of 128 called one after another.  us per chunk.

    python scripts/bench_fc_infer.py [--reps 5]
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
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--features", type=int, default=26 ** 3 * 64)
    ap.add_argument("--hidden", type=int, default=128)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    M, K, N = a.batch, a.features, a.hidden
    Kn = _native.kernels()
    st = _native.stream(None)
    x = (torch.rand(M, K, device="cuda") < 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.01).to(torch.bfloat16)
    b = torch.zeros(N, device="cuda")
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    res = {"S_default": int(Kn.dense_splits(M, N, K))}
    for S in sorted({8, 16, 32, 64, 128, res["S_default"]}):
        part = torch.empty(S, M, N, device="cuda")
        res[f"fwd_S{S}"] = timeit(lambda: Kn.dense_fwd(x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(),
                                                        part.data_ptr(), M, N, K, S, 1, 0, st, [], 1), a.reps)
    R = 128
    Sr = int(Kn.dense_splits(R, N, K))
    part = torch.empty(Sr, R, N, device="cuda")
    xs = [x[i:i + R] for i in range(0, M, R)]
    ys = [y[i:i + R] for i in range(0, M, R)]

    def rows():
        for xi, yi in zip(xs, ys):
            Kn.dense_fwd(xi.data_ptr(), w.data_ptr(), b.data_ptr(), yi.data_ptr(), part.data_ptr(), R, N, K, Sr, 1, 0,
                         st, [], 1)
    res[f"fwd_rowblocks_{R}_S{Sr}"] = timeit(rows, a.reps)
    res["bytes_gb"] = round((x.numel() + w.numel()) * 2 / 1e9, 3)
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
