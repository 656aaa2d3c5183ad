#!/usr/bin/env python3
"""Headline benchmark: FeatureNet-3D training throughput (samples/s).

Metric / config from BASELINE.json: "samples/sec (64^3 voxel, 24-class) train
at 1/2/4/8 MI355X".  One training step = forward + backward + Adam update of
the full FeatureNet-3D (4 Conv3d+BN+ReLU, fused MaxPool3d, FC128, FC24) on a
per-GPU batch of synthetic 64^3 binary voxel grids with random labels and
random-init weights, bf16 compute / fp32 master weights.  Data parallel over
N GPUs = one process per GPU, RCCL all-reduce of gradient buckets overlapped
with backward (weak scaling: the per-GPU batch is fixed).

    python bench.py                       # 1 GPU, defaults
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 20 --warmup 5

``--impl torch`` runs the stock PyTorch-ROCm eager baseline (MIOpen + DDP) on
the same data for the first-party comparison recorded in BASELINE.md.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# measured first-party baseline: stock PyTorch-ROCm eager on 1x MI355X, same config (bf16
# autocast, channels-last, MIOpen find mode via torch.backends.cudnn.benchmark so MIOpen
# times its solvers and keeps the fastest): `python bench.py --impl torch --torch-find`,
# re-measured in round 3 on the same box and in the same call as the native bench
# (profiles/r3_bench_torch_same_box.log: 6,068 samples/s, 21.1 ms/step; native on that box
# 25,030, profiles/r3_bench_native_same_box.log; round 2: 6,100 on another box).  (Round 1 quoted 106.8 samples/s from MIOpen's
# no-find fallback path -- a pathological baseline, withdrawn.)  The reference itself
# publishes no number (BASELINE.json "published": {}).  vs_baseline = value / (this * n_gpus).
TORCH_BASELINE_SAMPLES_PER_S_PER_GPU = 6068.1


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=128, help="per-GPU batch")
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--classes", type=int, default=24)
    ap.add_argument("--impl", choices=["native", "torch"], default="native")
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--dist-backend", choices=["auto", "nccl", "gloo"], default="auto",
                    help="auto = nccl (RCCL) on GPUs, gloo on CPU; gloo on GPUs lets several ranks share one "
                         "card to exercise the data-parallel path on a 1-GPU box")
    ap.add_argument("--pool", type=int, default=4, help="distinct synthetic batches resident on device")
    ap.add_argument("--tiny", action="store_true", help="16^3 2-class plumbing config (not the headline)")
    ap.add_argument("--model", choices=["cls", "seg"], default="cls",
                    help="cls = FeatureNet-3D classifier (headline); seg = per-voxel segmentation head "
                         "(BASELINE config 4, 25 voxel classes)")
    ap.add_argument("--torch-layout", choices=["ndhwc", "ncdhw"], default="ndhwc",
                    help="memory format of the stock-PyTorch baseline (--impl torch)")
    ap.add_argument("--torch-amp", choices=["bf16", "off"], default="bf16",
                    help="stock-PyTorch baseline: bf16 autocast or plain fp32 (whichever MIOpen runs faster)")
    ap.add_argument("--torch-find", action="store_true",
                    help="stock-PyTorch baseline: torch.backends.cudnn.benchmark (MIOpen find: times every "
                         "applicable solver per shape during warmup and keeps the fastest)")
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                    help="native path: replay the whole training step (forward, backward, bucketed "
                         "all-reduce, Adam) as one captured hipGraph; auto = on for 1 rank and for RCCL "
                         "ranks (falls back to eager when any rank fails to capture)")
    ap.add_argument("--force-allreduce", action="store_true",
                    help="create the process group even at 1 rank and issue the bucketed all-reduces "
                         "(exercises the RCCL path from the gradient hooks on a 1-GPU box)")
    return ap.parse_args()


def _free_port() -> int:
    import socket

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _self_launch(n: int) -> int:
    """--gpus N > 1 without torchrun: run N ranks as CHILD processes (never exec; the
    parent has not touched the GPU) and return their exit code."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__),
           *sys.argv[1:]]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


def _peak_bf16_tflops(dev) -> float | None:
    """Dense bf16 MFMA peak of the device: CUs x 4 SIMDs x 1024 flop/clk x max clock."""
    if dev.type != "cuda":
        return None
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    mhz = 2400.0
    try:
        import subprocess

        out = subprocess.run(["rocminfo"], capture_output=True, text=True, timeout=30).stdout
        for blk in out.split("Agent ")[1:]:
            if "gfx950" in blk and "Max Clock Freq. (MHz):" in blk:
                mhz = float(blk.split("Max Clock Freq. (MHz):")[1].split()[0])
                break
    except Exception:  # noqa: BLE001 - rocminfo missing: use the gfx950 spec clock
        pass
    return cus * 4 * 1024 * mhz * 1e6 / 1e12


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_self_launch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch one rank per GPU")
    use_cuda = args.device == "cuda"
    backend = args.dist_backend if args.dist_backend != "auto" else ("nccl" if use_cuda else "gloo")
    if use_cuda:
        ndev = torch.cuda.device_count()
        if backend == "nccl" and world > ndev:
            raise SystemExit(f"bench.py: {world} RCCL ranks need {world} GPUs, {ndev} visible "
                             "(--dist-backend gloo lets ranks share a card)")
        gpu = local % max(1, ndev)   # ranks share a card only in gloo tests
        torch.cuda.set_device(gpu)
        dev = torch.device("cuda", gpu)
    else:
        dev = torch.device("cpu")
    if world > 1 or args.force_allreduce:
        from featurenet_amd.parallel.ddp import init_from_env

        if args.force_allreduce and world == 1:
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
        init_from_env(backend, force=args.force_allreduce)
    comm_world = dist.get_world_size() if dist.is_initialized() else 1
    assert comm_world == world, (comm_world, world)

    torch.manual_seed(1234 + rank)
    if args.tiny:
        args.size, args.classes = 16, 2
    B, S, NC = args.batch, args.size, args.classes
    # synthetic 64^3 occupancy grids (~30% filled) + random labels, device resident
    # binary voxel occupancy: uint8 on the native path (the space-to-depth stem reads the bytes --
    # a quarter of the copy-in and stem-packing traffic; 0 / 1 are exact in either type)
    vox = torch.uint8 if args.impl == "native" and dev.type == "cuda" else torch.bfloat16
    xs = [(torch.rand(B, S, S, S, 1, device=dev) < 0.3).to(vox) for _ in range(args.pool)]
    if args.model == "seg":
        NC = 25
        # per-voxel class labels as bytes (25 classes): an eighth of int64's bytes to copy in and read
        ys = [torch.randint(0, NC, (B, S, S, S), device=dev, dtype=torch.uint8) for _ in range(args.pool)]
    else:
        ys = [torch.randint(0, NC, (B,), device=dev) for _ in range(args.pool)]

    if args.impl == "native":
        from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig
        from featurenet_amd.ops import FlatAdam, softmax_xent
        from featurenet_amd.ops.loss import backward as loss_backward   # (unit-seeded: no fill launch)
        from featurenet_amd.parallel.ddp import GradBucketer
        from featurenet_amd.training.flat import FlatParams

        torch.manual_seed(1234)  # identical init on every rank (also broadcast below)
        cfg = FeatureNet3DConfig.tiny() if args.tiny else FeatureNet3DConfig(input_size=S, num_classes=NC)
        if args.model == "seg":
            from featurenet_amd.models.featurenet3d import FeatureNet3DSeg

            model = FeatureNet3DSeg(input_size=S, num_classes=NC, widths=cfg.widths).to(dev)
        else:
            model = FeatureNet3D(cfg).to(dev)
        flat = FlatParams(model)
        opt = FlatAdam(flat.data, flat.grad, lr=1e-3)
        bucketer = GradBucketer(flat, bucket_mb=args.bucket_mb, force=args.force_allreduce)
        bucketer.broadcast_from(0)

        def loss_of(x, y):
            # the model's own loss where it has one (the segmentation head computes the per-voxel
            # cross-entropy in its epilogue: no logits tensor), else softmax_xent of the logits
            return model.loss(x, y) if hasattr(model, "loss") else softmax_xent(model(x), y)

        def step(i):
            flat.zero_grad()
            loss = loss_of(xs[i % args.pool], ys[i % args.pool])
            loss_backward(loss)
            scale = bucketer.finish()
            opt.step(grad_scale=scale)
            return loss
        graph_on = use_cuda and (args.graph == "on" or (args.graph == "auto" and backend != "gloo"))
        if graph_on:
            opt.enable_device_state()
            opt.sync_device_state(grad_scale=1.0 / world if bucketer.active else 1.0)
        model_name = "FeatureNet-3D" if args.model == "cls" else "FeatureNet-3D-Seg (per-voxel head)"
        flops = model.train_flops_per_sample() if hasattr(model, "train_flops_per_sample") else None
    else:
        graph_on = False
        from bench.torch_baseline import TorchFeatureNet3D

        if args.torch_find:
            torch.backends.cudnn.benchmark = True
        bucketer = None
        torch.manual_seed(1234)
        model = TorchFeatureNet3D(input_size=S, num_classes=NC).to(dev)
        cl = use_cuda and args.torch_layout == "ndhwc"
        if cl:
            model = model.to(memory_format=torch.channels_last_3d)
        dmodel = model
        if world > 1:
            dmodel = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local] if use_cuda else None)
        opt = torch.optim.Adam(model.parameters(), lr=1e-3)
        xs = [x.permute(0, 4, 1, 2, 3) for x in xs]  # NCDHW view of the channels-last data
        xs = [x.contiguous(memory_format=torch.channels_last_3d) if cl else x.contiguous() for x in xs]
        lossf = torch.nn.CrossEntropyLoss()

        def step(i):
            opt.zero_grad(set_to_none=True)
            with torch.autocast(device_type="cuda" if use_cuda else "cpu", dtype=torch.bfloat16,
                                enabled=args.torch_amp == "bf16"):
                logits = dmodel(xs[i % args.pool].float() if args.torch_amp == "off" else xs[i % args.pool])
            loss = lossf(logits.float(), ys[i % args.pool])
            loss.backward()
            opt.step()
            return loss
        model_name = f"FeatureNet-3D (stock PyTorch eager baseline, {args.torch_layout}, amp={args.torch_amp})"
        flops = None

    def sync():
        if use_cuda:
            torch.cuda.synchronize()
        if dist.is_initialized():
            dist.barrier()

    for i in range(args.warmup):
        step(i)
    sync()
    if args.impl == "native" and dist.is_initialized():
        from featurenet_amd.ops import tuning

        tuning.sync_from_rank0()      # every rank runs rank 0's per-shape kernels (deterministic table)
    graph_used = False
    graph_fallback = False
    if graph_on:
        # capture one step on static input buffers (the eager warmup above already ran the
        # per-shape kernel selection); every timed step = copy the batch in + one replay
        from featurenet_amd import _native

        sx, sy = xs[0].clone(), ys[0].clone()
        g = torch.cuda.CUDAGraph()
        ok = True
        try:
            with torch.cuda.graph(g):
                flat.zero_grad()
                gl = loss_of(sx, sy)
                loss_backward(gl)
                bucketer.finish()
                opt.step_device()
        except Exception as ex:  # noqa: BLE001 - report and fall back to eager steps
            print(f"bench.py rank {rank}: step capture failed, eager steps: {ex}", file=sys.stderr)
            bucketer.reset()
            ok = False
        if dist.is_initialized():
            f = torch.tensor([1.0 if ok else 0.0], device=dev if backend == "nccl" else "cpu")
            dist.all_reduce(f, op=dist.ReduceOp.MIN)
            ok = bool(f.item() > 0.5)
        graph_fallback = not ok
        if ok:
            graph_used = True

            def step(i):
                _native.copy_in(sx, xs[i % args.pool], sy, ys[i % args.pool])   # (one launch)
                g.replay()
                opt.t += 1
                return gl
        sync()
    t0 = time.perf_counter()
    loss = None
    for i in range(args.steps):
        loss = step(args.warmup + i)
    sync()
    elapsed = time.perf_counter() - t0
    rank_ms = None
    if dist.is_initialized():
        tdev = dev if backend == "nccl" else "cpu"
        ts = [torch.zeros(1, device=tdev, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(ts, torch.tensor([elapsed], device=tdev, dtype=torch.float64))
        per = [float(t.item()) for t in ts]
        elapsed = max(per)                     # the job's time is the slowest rank's
        rank_ms = [round(v / max(args.steps, 1) * 1e3, 3) for v in per]
    # communication diagnostics, measured AFTER the timed region: the bucketed
    # all-reduce of the whole gradient on its own (what the overlap has to hide)
    allreduce_ms = None
    n_buckets = None
    if bucketer is not None:
        n_buckets = bucketer.n_buckets
        if bucketer.active:
            allreduce_ms = bucketer.time_allreduce()
    peak = _peak_bf16_tflops(dev)
    ms = elapsed / max(args.steps, 1) * 1e3
    value = args.steps * B * world / elapsed
    base = TORCH_BASELINE_SAMPLES_PER_S_PER_GPU
    same_cfg = args.batch == 128 and args.size == 64 and args.classes == 24 and not args.tiny and args.model == "cls"
    vs = (value / (base * world)) if base and same_cfg else None
    if rank == 0:
        out = {
            "metric": (f"samples/sec ({S}^3 voxel, {NC}-class) train" if args.model == "cls"
                       else f"samples/sec ({S}^3 voxel, per-voxel segmentation) train"),
            "value": round(value, 2),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None if vs is None else round(vs, 3),
            "dtype": "fp32" if (not use_cuda or (args.impl == "torch" and args.torch_amp == "off")) else "bf16",
            "data": f"synthetic (random {args.size}^3 binary voxels{' stored as uint8' if xs[0].dtype == torch.uint8 else ''}, "
                    f"random labels, random-init weights)",
            "config": {
                "model": model_name,
                "global_batch": B * world,
                "per_gpu_batch": B,
                "seq_len": None,
                "input": f"{S}^3x1 voxels",
                "classes": NC,
                "parallelism": f"dp{world}",
                "impl": args.impl,
                "optimizer": "adam", "graph": graph_used,
            },
            "graph_fallback": graph_fallback,
            "final_loss": None if loss is None else round(float(loss.detach()), 4),
        }
        out["dist"] = {
            "backend": backend if dist.is_initialized() else None,
            "rccl_world": comm_world if dist.is_initialized() and backend == "nccl" else None,
            "buckets": n_buckets,
            "bucket_mb": args.bucket_mb,
            "allreduce_ms": None if allreduce_ms is None else round(allreduce_ms, 3),
            "forced_single_rank": bool(args.force_allreduce and world == 1),
            "rank_ms_per_step": rank_ms,
            "rank_spread_pct": None if not rank_ms else round(100.0 * (max(rank_ms) - min(rank_ms)) / max(rank_ms), 2),
        }
        if flops:
            out["model_tflops_per_s"] = round(flops * value / 1e12, 2)
            if peak:
                # whole-job model FLOP/s over the job's aggregate dense bf16 MFMA peak
                out["pct_bf16_peak"] = round(100.0 * flops * value / 1e12 / (peak * world), 2)
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
