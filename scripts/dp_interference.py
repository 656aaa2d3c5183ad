#!/usr/bin/env python3
"""How the training step degrades when other kernels hold CUs -- the one-GPU stand-in for the
RCCL ring kernels that overlap backward in data-parallel training (an 8-GPU ring all-reduce
runs its channels as workgroups on the same CUs as the conv kernels).

A side stream runs ``cu_occupy`` (csrc/kernels/misc.hip): N workgroups spinning for the whole
step, each holding ``--lds`` bytes of LDS (> 80 KB: one occupier per CU, and no big-tile conv workgroup fits next to it,
so the CU is lost to the conv for the spin; 0: the CU is shared, only issue slots are taken).
The main stream replays the captured FeatureNet-3D training step (as bench.py: forward, backward,
Adam; 64^3, batch 128).  Printed: median step time per N, and the stretch over N = 0.

    python scripts/dp_interference.py --cus 0 8 16 32 --lds 98304 0
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cus", type=int, nargs="+", default=[0, 8, 16, 32])
    ap.add_argument("--lds", type=int, nargs="+", default=[98304, 0])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--spin-us", type=int, default=0, help="occupier spin (0: 1.2 x the quiet step)")
    ap.add_argument("--phase", choices=["step", "backward"], default="step",
                    help="step: the occupier starts with the step; backward: it starts after the forward's "
                         "share of the step (measured quiet), the way the first RCCL bucket starts")
    args = ap.parse_args()

    from featurenet_amd import _native
    from featurenet_amd.models.featurenet3d import FeatureNet3D
    from featurenet_amd.ops import FlatAdam, softmax_xent
    from featurenet_amd.ops.loss import backward as loss_backward
    from featurenet_amd.training.flat import FlatParams

    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    B = args.batch
    x = (torch.rand(B, 64, 64, 64, 1, device=dev) < 0.3).to(torch.uint8)
    y = torch.randint(0, 24, (B,), device=dev)
    model = FeatureNet3D().to(dev)
    flat = FlatParams(model)
    opt = FlatAdam(flat.data, flat.grad, lr=1e-3)
    for _ in range(3):
        flat.zero_grad()
        loss_backward(softmax_xent(model(x), y))
        opt.step()
    torch.cuda.synchronize()
    opt.enable_device_state()
    opt.sync_device_state(grad_scale=1.0)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        flat.zero_grad()
        loss_backward(softmax_xent(model(x), y))
        opt.step_device()
    # forward-only graph: the forward's share of the step (for --phase backward)
    gf = torch.cuda.CUDAGraph()
    with torch.no_grad(), torch.cuda.graph(gf):
        model(x)
    K = _native.kernels()
    sink = torch.zeros(1024, dtype=torch.int32, device=dev)
    side = torch.cuda.Stream(dev)
    main_s = torch.cuda.current_stream(dev)

    def timed(fn, n):
        ts = []
        for _ in range(n):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(main_s)
            fn()
            e1.record(main_s)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        return ts[len(ts) // 2]

    for _ in range(5):
        g.replay()
    quiet = timed(g.replay, args.steps)
    fwd = timed(gf.replay, args.steps)
    spin = args.spin_us or int(quiet * 1e3 * 1.2)
    print(f"[interference] quiet step {quiet:.3f} ms, forward {fwd:.3f} ms, spin {spin} us", flush=True)
    rows = []
    for lds in args.lds:
        for n in args.cus:
            def run():
                if n:
                    if args.phase == "backward":
                        # start the occupier when the step's forward is about done: a side-stream
                        # delay of the forward's time (a first spin with no CUs to speak of)
                        with torch.cuda.stream(side):
                            K.cu_occupy(1, int(fwd * 1e3), 0, sink.data_ptr(), side.cuda_stream)
                            K.cu_occupy(n, spin, lds, sink.data_ptr(), side.cuda_stream)
                    else:
                        K.cu_occupy(n, spin, lds, sink.data_ptr(), side.cuda_stream)
                g.replay()
            t = timed(run, args.steps)
            r = {"occupied_cus": n, "lds": lds, "phase": args.phase, "step_ms": round(t, 3),
                 "stretch_pct": round(100.0 * (t / quiet - 1.0), 2),
                 "cu_share_pct": round(100.0 * n / torch.cuda.get_device_properties(dev).multi_processor_count, 2)}
            rows.append(r)
            print(json.dumps(r), flush=True)
    torch.cuda.synchronize()
    assert int(sink.sum()) == 0


if __name__ == "__main__":
    main()
