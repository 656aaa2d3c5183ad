"""The RCCL data-parallel path on one GPU: a single-rank ProcessGroupNCCL (= RCCL) communicator.

RCCL refuses two ranks on one device, so the multi-rank collective itself is the driver's
8-GPU run.  What one GPU can check is everything around it, at the headline shapes
(FeatureNet-3D, 64^3, batch 128):

* the gradient hooks issue every bucket's ``all_reduce`` during backward (eager, and while a
  hipGraph captures the whole step -- forward, backward, bucketed all-reduce, Adam);
* a step with the collectives gives the same loss, gradients and updated weights, bit for bit,
  as the same step without them (a one-rank sum is the identity; nothing else may change), and
  so does the graph replay of the captured step;
* ``bench.py --force-allreduce`` -- the driver's exact entry point -- captures the step with the
  RCCL collectives in it (no eager fallback) and issues all buckets.

Reference anchor: ``/root/reference/model/keras_model.py:137-146`` (``multi_gpu_model`` with a
silent single-GPU fallback; here a capture failure is reported, see ``graph_fallback``).
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _worker(rank, tmp, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    import torch.distributed as dist

    from featurenet_amd.models.featurenet3d import FeatureNet3D
    from featurenet_amd.ops import FlatAdam, softmax_xent
    from featurenet_amd.ops.loss import backward as loss_backward
    from featurenet_amd.parallel.ddp import GradBucketer, init_from_env
    from featurenet_amd.training.flat import FlatParams

    init_from_env("nccl", force=True)
    res = {}
    try:
        assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
        dev = torch.device("cuda", 0)
        torch.manual_seed(21)
        model = FeatureNet3D().to(dev)
        flat = FlatParams(model)
        opt = FlatAdam(flat.data, flat.grad, lr=1e-3)
        opt.enable_device_state(grad_scale=1.0)          # every step below: the device-state Adam
        b = GradBucketer(flat, bucket_mb=32.0, force=True)
        assert b.active and b.n_buckets >= 3, b.n_buckets
        res["n_buckets"] = b.n_buckets
        x = (torch.rand(128, 64, 64, 64, 1, device=dev) < 0.3).to(torch.uint8)
        y = torch.randint(0, 24, (128,), device=dev)

        def step():
            flat.zero_grad()
            loss = softmax_xent(model(x), y)
            loss_backward(loss)
            scale = b.finish()
            opt.step(grad_scale=scale)
            return loss

        b.paused = True
        for _ in range(2):                                 # warmup: per-shape kernel selection
            step()
        torch.cuda.synchronize()
        bufs = list(model.buffers())
        snap = [flat.data.clone(), opt.m.clone(), opt.v.clone(), opt._dev[1].clone()] + [t.clone() for t in bufs]
        t_host = opt.t

        def restore():
            for dst, src in zip([flat.data, opt.m, opt.v, opt._dev[1]] + bufs, snap):
                dst.copy_(src)
            opt.t = t_host
            torch.cuda.synchronize()

        def outcome(loss):
            torch.cuda.synchronize()
            return (loss.detach().float().cpu().clone(), flat.grad.cpu().clone(), flat.data.cpu().clone(),
                    opt.m.cpu().clone())

        restore()
        ref = outcome(step())                              # no collectives
        restore()
        b.paused = False
        n0 = b.n_collectives
        eager = outcome(step())                            # hook-issued single-rank all-reduces
        res["eager_collectives"] = b.n_collectives - n0
        restore()
        g = torch.cuda.CUDAGraph()
        n0 = b.n_collectives
        with torch.cuda.graph(g):
            flat.zero_grad()
            gl = softmax_xent(model(x), y)
            loss_backward(gl)
            b.finish()
            opt.step_device()
        res["captured_collectives"] = b.n_collectives - n0
        restore()
        g.replay()
        graph = outcome(gl)
        names = ("loss", "grad", "weights", "adam_m")
        res["eager_vs_ref"] = [n for n, a, c in zip(names, eager, ref) if not torch.equal(a, c)]
        res["graph_vs_ref"] = [n for n, a, c in zip(names, graph, ref) if not torch.equal(a, c)]
        res["grad_norm"] = float(ref[1].norm())
        res["loss"] = float(ref[0])
    finally:
        with open(os.path.join(tmp, "res.json"), "w") as f:
            json.dump(res, f)
        dist.destroy_process_group()


def test_single_rank_rccl_step_bitwise_equal_to_local_step(tmp_path):
    from featurenet_amd import _native

    assert _native.kernels_available(), "HIP kernel library (_C) must be built and loadable on the GPU box"
    mp.start_processes(_worker, args=(str(tmp_path), _free_port()), nprocs=1, start_method="spawn")
    r = json.loads((tmp_path / "res.json").read_text())
    print(r)
    assert r["eager_collectives"] == r["n_buckets"], r
    assert r["captured_collectives"] == r["n_buckets"], r
    assert r["grad_norm"] > 0 and r["loss"] == r["loss"], r
    assert r["eager_vs_ref"] == [], r
    assert r["graph_vs_ref"] == [], r


def test_bench_force_allreduce_captures_rccl_step(tmp_path):
    """The driver's entry point with a single-rank RCCL communicator: hipGraph capture with the
    hook-issued collectives inside, no eager fallback, every bucket issued."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--force-allreduce", "--steps", "5",
                        "--warmup", "3"], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    print(line)
    assert out["config"]["graph"] is True and out["graph_fallback"] is False, out
    d = out["dist"]
    assert d["backend"] == "nccl" and d["rccl_world"] == 1 and d["forced_single_rank"] is True, d
    assert d["buckets"] >= 3 and d["allreduce_ms"] is not None and d["allreduce_ms"] > 0, d
    assert out["value"] > 0 and out["final_loss"] == out["final_loss"], out
