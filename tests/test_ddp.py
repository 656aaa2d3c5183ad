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


_BN_CFG = dict(input_size=16, num_classes=4, widths=(8, 8, 16, 16), kernels=(3, 3, 3, 3), strides=(1, 1, 1, 1),
               fc=16)


def _bn_shards(n=8, seed=5):
    g = torch.Generator().manual_seed(seed)
    x = (torch.rand(WORLD * n, 16, 16, 16, 1, generator=g) < 0.3).float()
    x[n:] *= 2.0                      # the two shards have different statistics
    return x, torch.randint(0, 4, (WORLD * n,), generator=g)


def _precise_bn_worker(rank, tmp):
    dist.init_process_group("gloo", init_method=f"file://{tmp}/rdzv", rank=rank, world_size=WORLD)
    try:
        from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig
        from featurenet_amd.training.trainer import Trainer

        torch.manual_seed(rank)
        tr = Trainer(FeatureNet3D(FeatureNet3DConfig(**_BN_CFG)), lr=1e-3, device="cpu")
        x, y = _bn_shards()
        # the trainer shards x by rank itself (strided slice of a global permutation); one
        # full-shard batch per rank
        used = tr.recalibrate_bn(x, y, batches=1, batch_size=len(x) // WORLD)
        assert used == 1
        torch.save({k: v.clone() for k, v in tr.model.state_dict().items()}, f"{tmp}/bn{rank}.pt")
    finally:
        dist.destroy_process_group()


def test_precise_bn_averages_running_stats_across_ranks(tmp_path):
    """PreciseBN under DP: every replica ends with the mean over ranks of its shard's batch statistics."""
    from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig
    from featurenet_amd.training.trainer import bn_modules

    mp.start_processes(_precise_bn_worker, args=(str(tmp_path),), nprocs=WORLD, start_method="spawn")
    sd = [torch.load(tmp_path / f"bn{r}.pt", weights_only=True) for r in range(WORLD)]
    for k in sd[0]:
        assert torch.equal(sd[0][k], sd[1][k]), k           # replicas agree (weights broadcast, stats reduced)
    # expected: the same model, momentum 1, one train-mode forward per shard, averaged
    x, yy = _bn_shards()
    n = len(x) // WORLD
    per_rank = []
    from featurenet_amd.training.data import DeviceLoader

    for r in range(WORLD):
        # rank r's batch: its strided slice of the recalibration loader's global permutation
        idx = DeviceLoader(x, yy, n, "cpu", rank=r, world=WORLD, seed=7919).indices(0)
        m = FeatureNet3D(FeatureNet3DConfig(**_BN_CFG))
        m.load_state_dict(sd[0])
        mods = bn_modules(m)
        for mod, attr in mods:
            setattr(mod, attr, 1.0)
        m.train()
        with torch.no_grad():
            m(x[idx])
        per_rank.append([(mod.running_mean.clone(), mod.running_var.clone()) for mod, _ in mods])
    m = FeatureNet3D(FeatureNet3DConfig(**_BN_CFG))
    m.load_state_dict(sd[0])
    for i, (mod, _) in enumerate(bn_modules(m)):
        exp_mean = (per_rank[0][i][0] + per_rank[1][i][0]) / 2
        exp_var = (per_rank[0][i][1] + per_rank[1][i][1]) / 2
        torch.testing.assert_close(mod.running_mean, exp_mean, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(mod.running_var, exp_var, rtol=1e-4, atol=1e-5)
        assert not torch.allclose(per_rank[0][i][0], per_rank[1][i][0])   # shards really differ


# ---------------------------------------------------------------- bucket planning
def test_plan_buckets_closes_before_overflow_and_isolates_large_tensors():
    from featurenet_amd.parallel.ddp import plan_buckets

    # cap 100: 10+30+49 fits (89); 20 would overflow -> new bucket; 60 >= cap/2 -> alone
    assert plan_buckets([10, 30, 49, 20, 60, 5, 5], 100) == [[0, 1, 2], [3], [4], [5, 6]]
    assert plan_buckets([200], 100) == [[0]]
    assert plan_buckets([1] * 5, 4) == [[0, 1, 2, 3], [4]]
    for sizes in ([3, 7, 1, 90, 45, 2, 60, 1], [1] * 50, [49, 51, 49, 51]):
        plan = plan_buckets(sizes, 100)
        assert [i for b in plan for i in b] == list(range(len(sizes)))      # order kept, all covered
        for b in plan:
            assert len(b) == 1 or sum(sizes[i] for i in b) <= 100


def test_plan_buckets_tail_split_survives_a_large_last_tensor():
    """a last gradient larger than the tail cap (or than cap/2) must not switch the
    tail split off: it gets a bucket of its own and the walk continues with small caps."""
    from featurenet_amd.parallel.ddp import plan_buckets

    sizes = [40, 40, 40, 10, 10, 10, 10, 10, 10, 70]
    plan = plan_buckets(sizes, 100, tail_cap=10)
    assert [i for b in plan for i in b] == list(range(len(sizes)))
    assert plan[-1] == [9]                         # the large last tensor alone
    assert plan[-2] == [8]                         # then tail buckets of 10, 20, 40, ...
    assert plan[-3] == [6, 7]
    assert all(len(b) == 1 or sum(sizes[i] for i in b) <= 100 for b in plan)
    # a last tensor just above the tail cap still starts the tail at the tail cap
    plan = plan_buckets([5] * 20 + [30], 100, tail_cap=8)
    assert plan[-1] == [20] and plan[-2] == [17, 18, 19]


def test_featurenet3d_fc1_gradient_has_its_own_bucket():
    """at the default 32 MiB cap FC1's 32.8 MB weight gradient must not share a
    bucket with conv gradients (it is ready first; the convs come much later in backward)."""
    from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig
    from featurenet_amd.parallel.ddp import GradBucketer
    from featurenet_amd.training.flat import FlatParams

    m = FeatureNet3D(FeatureNet3DConfig())
    flat = FlatParams(m)
    b = GradBucketer(flat, bucket_mb=32.0)
    names = {id(p): n for n, p in m.named_parameters()}
    groups = [[names[id(p)] for p in ps] for ps in b.members]
    fc1 = [g for g in groups if "fc1.weight" in g]
    assert len(fc1) == 1 and not any(n.startswith("convs.") for n in fc1[0]), groups
    assert groups.index(fc1[0]) <= 1                              # issued at the start of backward
    conv_buckets = [g for g in groups if any(n.startswith("convs.") for n in g)]
    assert conv_buckets and all(not any(n.startswith("fc") for n in g) for g in conv_buckets)
    # buckets tile the flat buffer contiguously
    assert b.buckets[0][0] == 0 and b.buckets[-1][1] == flat.numel
    assert all(b.buckets[i][1] == b.buckets[i + 1][0] for i in range(len(b.buckets) - 1))


# ---------------------------------------------------------------- failure detection
def test_killed_rank_fails_fast(tmp_path):
    """A rank that dies mid-job makes the survivor exit non-zero (DistributedFailure)
    well inside the process-group timeout instead of hanging."""
    import socket
    import subprocess
    import sys
    import time

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    worker = os.path.join(os.path.dirname(__file__), "dp_fault_worker.py")
    procs = []
    t0 = time.time()
    for r in range(WORLD):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(WORLD), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), FN_PG_TIMEOUT="60", FN_KILL_RANK="1", OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, worker], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=150)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise AssertionError("a surviving rank hung after its peer died")
    elapsed = time.time() - t0
    assert procs[1].returncode == 17
    assert procs[0].returncode == 3, outs[0][-2000:]
    assert "DistributedFailure" in outs[0]
    assert elapsed < 120


def test_process_group_has_explicit_timeout(monkeypatch):
    from datetime import timedelta

    from featurenet_amd.parallel import ddp

    seen = {}

    def fake_init(backend, **kw):
        seen.update(kw, backend=backend)

    monkeypatch.setattr(ddp.dist, "is_initialized", lambda: False)
    monkeypatch.setattr(ddp.dist, "init_process_group", fake_init)
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("FN_PG_TIMEOUT", "42")
    ddp.init_from_env("gloo")
    assert seen["backend"] == "gloo" and seen["timeout"] == timedelta(seconds=42)


def test_tail_buckets_split_the_conv_gradients():
    """The gradients backward produces last are cut from the end into small buckets
    (0.25, 0.5, 1 MiB ...): FeatureNet-3D's stem, conv2 and conv3+conv4 reduce separately, so
    conv2's all-reduce overlaps the stem's weight gradient and only the stem's is exposed."""
    from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig
    from featurenet_amd.parallel.ddp import GradBucketer, plan_buckets
    from featurenet_amd.training.flat import FlatParams

    assert plan_buckets([5, 5, 40, 3, 4, 2, 1], 100, tail_cap=4) == [[0, 1], [2], [3, 4], [5, 6]]
    assert plan_buckets([5, 5, 40, 3, 4, 2, 1], 100, tail_cap=32) == [[0, 1, 2], [3, 4, 5, 6]]
    assert plan_buckets([5, 5, 50, 3, 4, 2, 1], 100, tail_cap=4) == [[0, 1], [2], [3, 4], [5, 6]]
    for sizes in ([3, 7, 1, 90, 45, 2, 60, 1], [1] * 50, [49, 51, 49, 51]):
        plan = plan_buckets(sizes, 100, tail_cap=8)
        assert [i for b in plan for i in b] == list(range(len(sizes)))
    m = FeatureNet3D(FeatureNet3DConfig())
    flat = FlatParams(m)
    b = GradBucketer(flat, bucket_mb=32.0)
    names = {id(p): n for n, p in m.named_parameters()}
    groups = [[names[id(p)] for p in ps] for ps in b.members]
    assert groups[-1] == ["convs.0.beta", "convs.0.gamma", "convs.0.weight"], groups
    assert groups[-2] == ["convs.1.beta", "convs.1.gamma", "convs.1.weight"], groups
    assert all(n.startswith(("convs.2", "convs.3")) for n in groups[-3]), groups


def _select_worker(rank, tmp):
    dist.init_process_group("gloo", init_method=f"file://{tmp}/rdzv", rank=rank, world_size=WORLD)
    try:
        from featurenet_amd.ops import tuning

        tuning._DECIDED.clear()
        # rank 1 decided differently (e.g. an autotuned timing); rank 0's decisions win
        tuning._DECIDED[("fwd", (1, 2, 3))] = rank == 0
        tuning._DECIDED[("wgrad", (4, 5, 6))] = rank != 0
        n = tuning.sync_from_rank0()
        torch.save({"n": n, "d": sorted(tuning.decisions().items())}, f"{tmp}/s{rank}.pt")
    finally:
        dist.destroy_process_group()


def test_kernel_choices_broadcast_from_rank0(tmp_path):
    """Every rank runs rank 0's per-shape kernel choice (identical kernels and rounding)."""
    import pickle  # noqa: F401 - (the files below are this test's own torch.save output)

    mp.start_processes(_select_worker, args=(str(tmp_path),), nprocs=WORLD, start_method="spawn")
    s = [torch.load(tmp_path / f"s{r}.pt", weights_only=False) for r in range(WORLD)]
    assert s[0]["d"] == s[1]["d"] == [(("fwd", (1, 2, 3)), True), (("wgrad", (4, 5, 6)), False)]


def test_kernel_selection_is_deterministic_without_timing(monkeypatch):
    """Default selection never times kernels: the table, then the rule (tile kernel)."""
    from featurenet_amd.ops import tuning
    from featurenet_amd.ops.spec import ConvSpec

    monkeypatch.delenv("FN_KERNEL_SELECT", raising=False)
    spec = ConvSpec.make((4, 11, 12, 13, 32), 32, 3)

    def boom():
        raise AssertionError("timed a kernel")

    tuning._DECIDED.pop(("fwd", tuning.shape_key(spec)), None)
    assert tuning.select("fwd", spec, boom, boom) is True
    monkeypatch.setitem(tuning.EXCEPTIONS, ("dgrad",) + tuning.shape_key(spec), False)
    tuning._DECIDED.pop(("dgrad", tuning.shape_key(spec)), None)
    assert tuning.select("dgrad", spec, boom, boom) is False
