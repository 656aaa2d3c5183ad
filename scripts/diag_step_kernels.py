#!/usr/bin/env python3
"""Which Python call launched each kernel of one eager FeatureNet-3D training step (the
headline bench's step: forward, backward, device-state Adam), in launch order: torch.profiler
with stacks, one line per kernel -- name, us, and the innermost featurenet_amd / bench frame.

    python scripts/diag_step_kernels.py [--batch 128] [--small-us 15]

Used to find the small launches of the step (fills, casts, scalar kernels) worth folding.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--small-us", type=float, default=1e9, help="list only kernels shorter than this")
    a = ap.parse_args()
    from featurenet_amd.models.featurenet3d import FeatureNet3D
    from featurenet_amd.ops import FlatAdam, softmax_xent
    from featurenet_amd.training.flat import FlatParams

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = FeatureNet3D().to(dev)
    flat = FlatParams(model)
    opt = FlatAdam(flat.data, flat.grad, lr=1e-3)
    opt.enable_device_state()
    opt.sync_device_state(grad_scale=1.0)
    x = (torch.rand(a.batch, 64, 64, 64, 1, device=dev) < 0.3).to(torch.bfloat16)
    y = torch.randint(0, 24, (a.batch,), device=dev)

    def step():
        flat.zero_grad()
        softmax_xent(model(x), y).backward()
        opt.step_device()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    # each kernel under the innermost op that launched it (its CPU event), in launch order
    evs = prof.profiler.function_events
    rows = []
    for e in evs:
        if not e.kernels:
            continue
        if any(c.kernels for c in e.cpu_children):
            continue                              # (a parent op: its children carry the kernels)
        stack = [s for s in (e.stack or []) if ("featurenet_amd" in s or "bench" in s or "scripts" in s)]
        where = stack[0] if stack else ""
        for k in e.kernels:
            rows.append((e.time_range.start, k.name, k.duration, e.name, where))
    rows.sort()
    tot = 0.0
    for _, name, dur, op, where in rows:
        tot += dur
        if dur < a.small_us:
            print(f"{dur:8.1f} us  {name[:60]:60s}  {op[:28]:28s}  {where}")
    print(f"kernels {len(rows)}, total {tot:.1f} us")


if __name__ == "__main__":
    main()
