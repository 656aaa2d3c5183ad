#!/usr/bin/env python3
"""How the training step degrades when other kernels hold CUs for a while -- the one-GPU stand-in
for the RCCL ring kernels of the data-parallel all-reduce, which run their channels as workgroups
on the same CUs as the backward's conv kernels (an 8-GPU ring all-reduce of a 32 MB bucket holds
its CUs for a few hundred microseconds).

Every step of a timed run of back-to-back graph replays (the captured FeatureNet-3D training step
of bench.py: forward, backward, Adam; 64^3, batch 128) gets a BURST on a side stream: once the
replay starts (an event on the main stream), a one-workgroup delay kernel spins ``offset`` us, then
``cu_occupy`` (csrc/kernels/misc.hip) runs N workgroups for ``--burst-us``, each holding ``--lds``
bytes of LDS (> 80 KB: one occupier per CU, and no big-tile conv workgroup fits next to it -- the
CU is lost to the conv kernels for the burst; 0: the CU is shared, only issue slots are taken).
The offsets sweep the step, so the burst lands on every kernel in turn; printed per (N, LDS): the
mean step time over the offsets and its stretch over the quiet step.

    python scripts/dp_interference.py --cus 0 8 16 32 --lds 98304 0 --burst-us 300
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
    ap.add_argument("--burst-us", type=int, default=300)
    ap.add_argument("--offsets", type=int, default=8, help="burst start points spread over the step")
    ap.add_argument("--reps", type=int, default=10, help="back-to-back steps per measurement")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--schedules", nargs="+", default=["static", "chunked"],
                    help="conv_tile BN-statistics schedules to measure (static: 1 GPU default; chunked: data parallel)")
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

    def capture():
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            flat.zero_grad()
            loss_backward(softmax_xent(model(x), y))
            opt.step_device()
        return g

    K = _native.kernels()
    sink = torch.zeros(1024, dtype=torch.int32, device=dev)
    side = torch.cuda.Stream(dev)
    main_s = torch.cuda.current_stream(dev)

    g = None

    def run(n, lds, off_us):
        evs = [torch.cuda.Event() for _ in range(args.reps)]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(main_s)
        for i in range(args.reps):
            if n:
                evs[i].record(main_s)
                side.wait_event(evs[i])
                if off_us:
                    K.cu_occupy(1, off_us, 0, sink.data_ptr(), side.cuda_stream)
                K.cu_occupy(n, args.burst_us, lds, sink.data_ptr(), side.cuda_stream)
            g.replay()
        e1.record(main_s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.reps

    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    for sched in args.schedules:
        K.conv_tile_set_schedule(1 if sched == "chunked" else 0)
        g = capture()
        for _ in range(3):
            run(0, 0, 0)
        quiet = sorted(run(0, 0, 0) for _ in range(5))[2]
        offs = [int(quiet * 1e3 * k / args.offsets) for k in range(args.offsets)]
        print(f"[interference] {sched}: quiet step {quiet:.3f} ms; burst {args.burst_us} us at offsets {offs} us",
              flush=True)
        for lds in args.lds:
            for n in args.cus:
                if n == 0:
                    continue
                per = [run(n, lds, o) for o in offs]
                mean = sum(per) / len(per)
                r = {"schedule": sched, "occupied_cus": n, "cu_share_pct": round(100.0 * n / ncu, 2), "lds": lds,
                     "burst_us": args.burst_us, "quiet_ms": round(quiet, 3), "step_ms_mean": round(mean, 3),
                     "step_ms_max": round(max(per), 3), "stretch_us_mean": round((mean - quiet) * 1e3, 1),
                     "stretch_pct": round(100.0 * (mean / quiet - 1.0), 2)}
                print(json.dumps(r), flush=True)
    K.conv_tile_set_schedule(-1)
    torch.cuda.synchronize()
    assert int(sink.sum()) == 0


if __name__ == "__main__":
    main()
