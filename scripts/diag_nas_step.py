#!/usr/bin/env python3
"""Kernels of one NAS candidate training step (the reference's lenet5 template at CIFAR shapes,
batch 64, Adam): the launch list of an eager step with the launching op, the kernel count, and
the graph-replay time per step.  One line per kernel, then a JSON summary line.

    python scripts/diag_nas_step.py [--template lenet5] [--batch 64] [--list]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--template", default="lenet5")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--list", action="store_true")
    ap.add_argument("--stacks", action="store_true", help="with --list: the package frames that launched torch glue")
    a = ap.parse_args()
    from featurenet_amd.ir.compile import compile_model
    from featurenet_amd.ir.parse import parse_feature_model
    from featurenet_amd.ops import FlatAdam, softmax_xent
    from featurenet_amd.ops.loss import backward as loss_backward
    from featurenet_amd.training.flat import FlatParams

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = compile_model(parse_feature_model(a.template, name="diag"), (32, 32, 3), 10).to(dev)
    flat = FlatParams(model)
    opt = FlatAdam(flat.data, flat.grad, lr=1e-3)
    opt.enable_device_state()
    opt.sync_device_state(grad_scale=1.0)
    x = torch.rand(a.batch, 32, 32, 3, device=dev)
    y = torch.randint(0, 10, (a.batch,), device=dev)

    def step():
        flat.zero_grad()
        loss_backward(softmax_xent(model(x), y))
        opt.step_device()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=a.stacks) as prof:
        step()
        torch.cuda.synchronize()
    rows = []
    for e in prof.profiler.function_events:
        # an op's own launches: a kernel a child op lists as well belongs to the child (the
        # native kernels of an autograd node with torch glue inside it are its own -- skipping
        # every op with a launching child dropped them)
        child = {(k.name, k.duration) for c in e.cpu_children for k in c.kernels}
        for k in e.kernels:
            if (k.name, k.duration) not in child:
                rows.append((e.time_range.start, k.name, k.duration, e.name, e))
    rows.sort(key=lambda r: r[0])
    if a.list:
        for _, name, dur, op, ev in rows:
            print(f"{dur:8.1f} us  {name[:70]:70s}  {op[:40]}")
            if a.stacks and op.startswith("aten::"):
                # (the launching op's nearest parents with a Python stack: the package frames)
                e2, fr = ev, []
                while e2 is not None and not fr:
                    fr = [f for f in (e2.stack or []) if "featurenet_amd" in f]
                    e2 = e2.cpu_parent
                for f in fr[:4]:
                    print(f"              <- {f}")
                if not fr:                        # (no Python stacks recorded: the op chain)
                    chain, e2 = [], ev.cpu_parent
                    while e2 is not None and len(chain) < 6:
                        chain.append(e2.name)
                        e2 = e2.cpu_parent
                    print(f"              <- {' <- '.join(chain)}")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    g.replay()
    torch.cuda.synchronize()
    reps = 200
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    print(json.dumps({"template": a.template, "batch": a.batch, "kernels_per_step": len(rows),
                      "kernel_us_eager": round(sum(r[2] for r in rows), 1), "graph_ms_per_step": round(ms, 4)}))


if __name__ == "__main__":
    main()
