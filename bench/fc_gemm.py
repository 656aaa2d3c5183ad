#!/usr/bin/env python3
"""FeatureNet-3D FC1 GEMM shapes on hipBLASLt: [B x F] x [F x 128] with F = 64000 (fwd), its dgrad and
wgrad, plus split-K (batched) variants of the skinny forward.  Prints one JSON line (us per call)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench.conv_kernels import timeit  # noqa: E402


def main():
    B, F, H = 128, 64000, 128
    x = torch.randn(B, F, device="cuda").to(torch.bfloat16)
    w = (torch.randn(H, F, device="cuda") * 0.01).to(torch.bfloat16)
    dy = torch.randn(B, H, device="cuda").to(torch.bfloat16)
    r = {}
    with torch.no_grad():
        r["fwd_matmul"] = timeit(lambda: torch.matmul(x, w.t()), 20)
        r["fwd_mm_f32out"] = timeit(lambda: torch.mm(x, w.t(), out_dtype=torch.float32), 20)
        for s in (4, 8, 16, 32):
            xs, ws = x.view(B, s, F // s).transpose(0, 1), w.view(H, s, F // s).permute(1, 2, 0)
            r[f"fwd_splitk{s}"] = timeit(lambda: torch.bmm(xs, ws).sum(0), 20)
        r["dgrad"] = timeit(lambda: torch.matmul(dy, w), 20)
        r["wgrad_bf16_then_f32"] = timeit(lambda: torch.matmul(dy.t(), x).float(), 20)
        r["wgrad_f32out"] = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32), 20)
        r["w_cast_bf16"] = timeit(lambda: w.float().to(torch.bfloat16), 20)
    print(json.dumps({k: round(v * 1e3, 1) for k, v in r.items()}), flush=True)


if __name__ == "__main__":
    main()
