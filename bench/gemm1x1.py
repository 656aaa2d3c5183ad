#!/usr/bin/env python3
"""1x1x1 conv (= plain GEMM over all voxels) timings: the streaming pointwise kernels (ConvFn fwd,
pw dgrad / wgrad), the generic implicit-GEMM kernels (native_*) and hipBLASLt
(torch.matmul) for the segmentation head shape [N*S^3, C] x [C, K].

    python bench/gemm1x1.py [--rows 33554432] [--cin 32] [--cout 25]
"""
import argparse
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench.conv_kernels import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=128 * 64 ** 3)
    ap.add_argument("--cin", type=int, default=32)
    ap.add_argument("--cout", type=int, default=25)
    a = ap.parse_args()
    C = importlib.import_module("featurenet_amd.ops.conv")
    from featurenet_amd.ops.spec import ConvSpec

    n = a.rows // (64 ** 3)
    x = torch.randn(n, 64, 64, 64, a.cin, device="cuda").to(torch.bfloat16)
    spec = ConvSpec.make(x.shape, a.cout, 1, 1)
    w = torch.randn(a.cout, 1, 1, 1, a.cin, device="cuda") * 0.1
    b = torch.zeros(a.cout, device="cuda")
    dy = torch.randn(spec.out_shape5, device="cuda").to(torch.bfloat16)
    x2, dy2, wb = x.reshape(-1, a.cin), dy.reshape(-1, a.cout), w.reshape(a.cout, a.cin).to(torch.bfloat16)
    res = {}
    with torch.no_grad():
        res["pointwise_fwd"] = timeit(lambda: C.ConvFn.apply(x, w, b, spec, 0, False), 10)
        res["blas_fwd"] = timeit(lambda: torch.addmm(b.to(torch.bfloat16), x2, wb.t()), 10)
        res["native_dgrad"] = timeit(lambda: C.native_conv_dgrad(dy, w, spec), 10)
        res["blas_dgrad"] = timeit(lambda: dy2 @ wb, 10)
        res["native_wgrad"] = timeit(lambda: C.native_conv_wgrad(dy, x, spec), 10)
        res["pointwise_dgrad"] = timeit(lambda: C.pw_fwd(dy2, w.reshape(a.cout, a.cin).t(), None, 0), 10)
        res["pointwise_wgrad"] = timeit(lambda: C.pw_wgrad(dy2, x2), 10)
        res["blas_wgrad"] = timeit(lambda: (dy2.t() @ x2).float(), 10)
        res["blas_wgrad_f32out"] = timeit(lambda: torch.mm(dy2.t(), x2, out_dtype=torch.float32), 10) \
            if "out_dtype" in torch.mm.__doc__ else None
    print(json.dumps({k: (round(v * 1e3, 1) if v is not None else None) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
