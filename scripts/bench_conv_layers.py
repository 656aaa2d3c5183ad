#!/usr/bin/env python3
"""Per-layer conv kernel timing for FeatureNet-3D at the headline batch.

For each stride-1 layer (conv2..conv4; ``--only seg_dec`` for the segmentation
decoder conv) times forward (BN-statistics epilogue) and dgrad on the big-tile
kernel (``conv_tile.hip``) and on the previous halo kernel (``conv_halo.hip``),
and the weight gradient on conv_halo and on the big-tile wgrad kernel (conv_wtile.hip), back to back on one stream (events around R
launches), and prints us/call and model TFLOP/s.

    python scripts/bench_conv_layers.py --batch 128 --reps 10
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import importlib  # noqa: E402

cv = importlib.import_module("featurenet_amd.ops.conv")   # the module (ops.conv is also a function name)
from featurenet_amd.ops import conv_tile as ct  # noqa: E402
from featurenet_amd.ops import conv_wtile as cw  # noqa: E402
from featurenet_amd.ops.spec import ConvSpec  # noqa: E402

LAYERS = [("stem_s2d", 32, 8, 32, 4, "valid"), ("conv2", 29, 32, 32, 5, "valid"), ("conv3", 25, 32, 64, 4, "valid"),
          ("conv4", 22, 64, 64, 3, "valid"), ("seg_dec", 64, 64, 32, 3, "same")]


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
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="")
    ap.add_argument("--tile-only", action="store_true", help="skip the conv_halo kernels")
    args = ap.parse_args()
    torch.manual_seed(0)
    rows = []
    for name, S, C, K, k, pad in LAYERS:
        if (args.only and name not in args.only.split(",")) or (not args.only and name == "seg_dec"):
            continue
        x = torch.randn(args.batch, S, S, S, C, device="cuda").to(torch.bfloat16)
        spec = ConvSpec.make(x.shape, K, k, 1, pad)
        w = torch.randn(K, k, k, k, C, device="cuda") * 0.05
        dy = torch.randn(spec.out_shape5, device="cuda").to(torch.bfloat16)
        gf = spec.flops() / 1e9
        pf, pd = ct.fwd_plan(spec), ct.dgrad_plan(spec)
        res = {"layer": name, "gflop": round(gf, 1), "tile_fwd_plan": str(pf), "tile_dgrad_plan": str(pd)}
        hf, hd, hw = cv.halo_fwd_plan(spec), cv.halo_dgrad_plan(spec), cv.halo_wgrad_plan(spec)
        pw = cw.plan(spec)
        # the training step's dgrad: the relu-mask statistics epilogue (static tile schedule)
        bits = (x.reshape(-1, 8) > 0).to(torch.uint8)
        mask = (bits * (2 ** torch.arange(8, device="cuda", dtype=torch.uint8))).sum(-1).to(torch.uint8).contiguous()
        mask_ok = pd is not None and ct.mask_dgrad_ok(pd, spec.C)
        runs = {"halo_fwd": (hf, lambda: cv.halo_conv_fwd(x, w, None, spec, 0, True, hf)),
                "tile_fwd": (pf, lambda: ct.conv_fwd(x, w, None, spec, 0, True, pf)),
                "halo_dgrad": (hd, lambda: cv.halo_conv_dgrad(dy, w, spec, hd)),
                "tile_dgrad": (pd, lambda: ct.conv_dgrad(dy, w, spec, pd)),
                "tile_dgrad_mask": (pd if mask_ok else None,
                                    lambda: ct.conv_dgrad(dy, w, spec, pd, bn=(x, None, 1, mask))),
                "halo_wgrad": (hw, lambda: cv.halo_conv_wgrad(dy, x, spec, hw)),
                "wtile_wgrad": (pw, lambda: cw.conv_wgrad(dy, x, spec, pw))}
        for kk, (pl, fn) in runs.items():
            if pl is None or (args.tile_only and kk.startswith("halo")):
                continue
            try:
                res[kk + "_us"] = round(timeit(fn, args.reps), 1)
            except RuntimeError as e:                # (e.g. no timing instance of this variant)
                res[kk + "_error"] = str(e).splitlines()[-1][:80]
                continue
            res[kk + "_tflops"] = round(gf / res[kk + "_us"] * 1e3, 1)
        rows.append(res)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
