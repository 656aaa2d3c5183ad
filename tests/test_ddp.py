"""Data-parallel path on CPU (gloo, world_size 2): bucketed all-reduce correctness.

The same code runs over RCCL on GPUs (backend "nccl"); here gloo checks that
the bucketed, hook-driven reductions produce exactly the single-process
average gradient and that replicas stay bit-identical through training.
"""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 2


def _model(seed=0):
    from featurenet_amd.ir.compile import compile_model
    from featurenet_amd.ir.parse import parse_feature_model

    torch.manual_seed(seed)
    return compile_model(parse_feature_model("lenet5", name="l"), (28, 28, 1), 10)


def _data(n=16, seed=1):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(n, 28, 28, 1, generator=g), torch.randint(0, 10, (n,), generator=g)


def _worker(rank, tmp, bucket_mb):
    dist.init_process_group("gloo", init_method=f"file://{tmp}/rdzv", rank=rank, world_size=WORLD)
    try:
        from featurenet_amd.ops import softmax_xent
        from featurenet_amd.training.trainer import Trainer

        torch.manual_seed(100 + rank)           # different init per rank: broadcast must fix it
        tr = Trainer(_model(seed=rank), lr=1e-3, device="cpu", bucket_mb=bucket_mb)
        assert len(tr.bucketer.buckets) > 1
        x, y = _data()
        xs, ys = x[rank::WORLD], y[rank::WORLD]
        tr.flat.zero_grad()
        loss, _ = softmax_xent(tr.model(xs), ys, 0.0, with_correct=True)
        loss.backward()
        scale = tr.bucketer.finish()
        torch.save({"grad": tr.flat.grad.clone() * scale, "data0": tr.flat.data.clone()}, f"{tmp}/g{rank}.pt")
        for _ in range(3):
            tr.train_step(xs, ys)
        torch.save({"data": tr.flat.data.clone()}, f"{tmp}/p{rank}.pt")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bucket_mb", [0.05, 0.5])
def test_bucketed_allreduce_matches_single_process(tmp_path, bucket_mb):
    mp.start_processes(_worker, args=(str(tmp_path), bucket_mb), nprocs=WORLD, start_method="spawn")
    g = [torch.load(tmp_path / f"g{r}.pt", weights_only=True) for r in range(WORLD)]
    p = [torch.load(tmp_path / f"p{r}.pt", weights_only=True) for r in range(WORLD)]
    # replicas start identical (broadcast from rank 0) and stay identical
    assert torch.equal(g[0]["data0"], g[1]["data0"])
    assert torch.equal(p[0]["data"], p[1]["data"])
    assert torch.equal(g[0]["grad"], g[1]["grad"])
    # single-process reference: average of the per-shard gradients
    from featurenet_amd.ops import softmax_xent
    from featurenet_amd.training.flat import FlatParams

    m = _model()
    flat = FlatParams(m)
    flat.data.copy_(g[0]["data0"])
    x, y = _data()
    acc = torch.zeros_like(flat.grad)
    for r in range(WORLD):
        flat.zero_grad()
        loss, _ = softmax_xent(m(x[r::WORLD]), y[r::WORLD], 0.0, with_correct=True)
        loss.backward()
        acc += flat.grad
    ref = acc * (1.0 / WORLD)
    torch.testing.assert_close(g[0]["grad"], ref, rtol=1e-6, atol=1e-8)
