"""Data-parallel data distribution (CPU, gloo): per-epoch global shuffling across replicas.

Reference: ``multi_gpu_model`` slices every batch of a Keras ``fit`` that reshuffles each
epoch (``/root/reference/model/keras_model.py:137-146``, ``helpers.py:103-111``), so every
replica sees a random cross-section of the data.  :class:`DeviceLoader` reproduces that
with one global permutation per epoch (shared seed) and rank-strided shards; these tests
run it on a CLASS-SORTED set (the order ``binvox_folder`` returns), where a fixed
contiguous shard per rank would give each rank only a few classes for the whole run.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLD = 8
NCLS = 24


def _sorted_set(per_class=8, size=28):
    y = np.repeat(np.arange(NCLS), per_class)                       # class-sorted, like binvox_folder
    x = np.zeros((len(y), size, size, 1), np.float32)
    x[:, 0, 0, 0] = np.arange(len(y))                               # sample id, recoverable from a batch
    return x, y


def test_loader_shards_partition_each_epoch_and_cover_every_class():
    from featurenet_amd.training.data import DeviceLoader

    x, y = _sorted_set()
    loaders = [DeviceLoader(x, y, 8, "cpu", rank=r, world=WORLD, seed=3) for r in range(WORLD)]
    prev = None
    for epoch in range(3):
        shards = []
        for ld in loaders:
            ld.set_epoch(epoch)
            ids = torch.cat([xb[:, 0, 0, 0] for xb, _ in ld]).long().tolist()
            labels = {int(y[i]) for i in ids}
            assert len(labels) >= NCLS // 2, (epoch, ld.rank, sorted(labels))   # (a contiguous shard: 3)
            shards.append(ids)
        flat = sorted(i for s in shards for i in s)
        assert flat == list(range(len(y))), "shards must partition the epoch"
        assert len({len(s) for s in shards}) == 1, "equal step counts per rank"
        if prev is not None:
            assert shards != prev, "shards must change between epochs"
        prev = shards
    # every rank sees EVERY class within an epoch on a large enough set
    x, y = _sorted_set(per_class=64)
    for r in range(WORLD):
        ld = DeviceLoader(x, y, 64, "cpu", rank=r, world=WORLD, seed=0)
        assert {int(y[i]) for i in ld.indices(0).tolist()} == set(range(NCLS))


def test_loader_uneven_tail_and_eval_mode():
    from featurenet_amd.training.data import DeviceLoader

    x, y = _sorted_set(per_class=3)          # 72 samples
    x, y = x[:70], y[:70]                    # 70 % 8 != 0
    tr = [DeviceLoader(x, y, 4, "cpu", rank=r, world=WORLD) for r in range(WORLD)]
    assert {len(ld.indices(0)) for ld in tr} == {70 // WORLD}
    ev = [DeviceLoader(x, y, 4, "cpu", rank=r, world=WORLD, shuffle=False, even=False) for r in range(WORLD)]
    got = sorted(i for ld in ev for i in ld.indices(0).tolist())
    assert got == list(range(70)), "evaluation shards cover every sample exactly once"


def _fit_worker(rank, tmp):
    dist.init_process_group("gloo", init_method=f"file://{tmp}/rdzv", rank=rank, world_size=WORLD)
    try:
        torch.set_num_threads(1)
        from featurenet_amd.ir.compile import compile_model
        from featurenet_amd.ir.parse import parse_feature_model
        from featurenet_amd.training.trainer import Trainer

        seen: dict = {}

        class Rec(Trainer):
            def train_step(self, xb, yb):
                seen.setdefault(self._ep, []).extend(xb[:, 0, 0, 0].long().tolist())
                return super().train_step(xb, yb)

        from featurenet_amd.training.callbacks import Callback

        class Ep(Callback):
            def on_epoch_begin(self, trainer, epoch):
                trainer._ep = epoch

        torch.manual_seed(0)
        model = compile_model(parse_feature_model("lenet5", name="l"), (28, 28, 1), NCLS)
        tr = Rec(model, lr=1e-3, device="cpu", precise_bn=0)
        x, y = _sorted_set(per_class=32)
        tr.fit(x, y, epochs=2, batch_size=8, callbacks=[Ep()], verbose=0, seed=5)
        with open(f"{tmp}/seen{rank}.json", "w") as f:
            json.dump({str(k): v for k, v in seen.items()}, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.slow
def test_fit_world8_gloo_global_shuffle(tmp_path):
    """Trainer.fit at world 8 on a class-sorted set: per-epoch union = the whole set, every
    rank gets a cross-section of the classes, shards change between epochs."""
    mp.start_processes(_fit_worker, args=(str(tmp_path),), nprocs=WORLD, start_method="spawn")
    _, y = _sorted_set(per_class=32)
    seen = [json.load(open(tmp_path / f"seen{r}.json")) for r in range(WORLD)]
    for ep in ("0", "1"):
        allids = sorted(i for s in seen for i in s[ep])
        assert allids == list(range(len(y)))
        for s in seen:
            assert len({int(y[i]) for i in s[ep]}) >= 20        # 96 draws of 24 classes
    assert [s["0"] for s in seen] != [s["1"] for s in seen]


@pytest.mark.slow
def test_bench_eight_ranks_gloo_json():
    """The driver's N=8 launch shape (one rank per GPU) rehearsed on the CPU with gloo."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", "29571", "bench.py", "--gpus", "8",
                        "--device", "cpu", "--dist-backend", "gloo", "--tiny", "--steps", "2", "--warmup", "1",
                        "--batch", "4"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 8 and r["config"]["parallelism"] == "dp8"
    assert r["config"]["global_batch"] == 4 * 8
    assert r["value"] == pytest.approx(32 / (r["ms_per_step"] / 1e3), rel=0.02)
    assert r["dist"]["rank_ms_per_step"] is not None and len(r["dist"]["rank_ms_per_step"]) == 8


def _resume_worker(rank, tmp, phase):
    dist.init_process_group("gloo", init_method=f"file://{tmp}/rdzv{phase}", rank=rank, world_size=2)
    try:
        torch.set_num_threads(1)
        from torch import nn

        from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig
        from featurenet_amd.ops.elementwise import dropout
        from featurenet_amd.training.callbacks import Callback
        from featurenet_amd.training.trainer import Trainer

        class Net(nn.Module):
            def __init__(self):
                super().__init__()
                self.body = FeatureNet3D(FeatureNet3DConfig.tiny())

            def forward(self, x):
                f = self.body.features(x).reshape(x.shape[0], -1)
                f = dropout(f, 0.3, self.training)      # torch's CPU generator: per rank
                return self.body.fc2(self.body.fc1(f), out_fp32=True)

        rs = np.random.RandomState(0)
        x = (rs.rand(64, 16, 16, 16) < 0.3).astype(np.float32)
        y = rs.randint(0, 2, 64).astype(np.int64)

        class SaveAt(Callback):
            def on_epoch_end(self, trainer, epoch, logs):
                if epoch == 1:
                    trainer.save(f"{tmp}/mid.fnk")

        torch.manual_seed(0)
        tr = Trainer(Net(), device="cpu", precise_bn=0)
        torch.manual_seed(1000 + 17 * rank + 31 * phase)  # per-rank dropout streams (and a different
        if phase == 0:                                    # one in the resumed process)
            tr.fit(x, y, epochs=4, batch_size=8, callbacks=[SaveAt()], verbose=0, seed=3)
        else:
            done = tr.resume(f"{tmp}/mid.fnk")
            assert done == 2
            tr.fit(x, y, epochs=4, batch_size=8, verbose=0, seed=3, initial_epoch=done)
        torch.save({"p": tr.flat.data.clone(), "loss": tr.history.history["loss"]}, f"{tmp}/r{rank}_{phase}.pt")
    finally:
        dist.destroy_process_group()


@pytest.mark.slow
def test_resume_world2_restores_each_ranks_generators(tmp_path):
    """Advisor r3: the checkpoint holds every rank's generator states (gathered, one writer);
    a 2-rank resumed run reproduces the uninterrupted one bit-for-bit."""
    mp.start_processes(_resume_worker, args=(str(tmp_path), 0), nprocs=2, start_method="spawn")
    from featurenet_amd.training.checkpoint import read_rng

    t, meta = read_rng(tmp_path / "mid.fnk")
    assert meta["world"] == 2 and "rank1.torch_cpu" in t
    assert not torch.equal(t["rank0.torch_cpu"], t["rank1.torch_cpu"])
    mp.start_processes(_resume_worker, args=(str(tmp_path), 1), nprocs=2, start_method="spawn")
    for r in range(2):
        a = torch.load(tmp_path / f"r{r}_0.pt", weights_only=True)
        b = torch.load(tmp_path / f"r{r}_1.pt", weights_only=True)
        assert a["loss"] == b["loss"], (a["loss"], b["loss"])
        assert torch.equal(a["p"], b["p"])


def _save_fail_worker(rank, tmp):
    dist.init_process_group("gloo", init_method=f"file://{tmp}/rdzv_save", rank=rank, world_size=2)
    try:
        torch.set_num_threads(1)
        from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig
        from featurenet_amd.training.trainer import Trainer

        torch.manual_seed(0)
        tr = Trainer(FeatureNet3D(FeatureNet3DConfig.tiny()), device="cpu", precise_bn=0)
        p = tr.save(f"{tmp}/ok.fnk")                     # every rank returns after the file exists
        assert os.path.exists(p) and os.path.getsize(p) > 0
        try:
            tr.save(f"{tmp}/ok.fnk/x.fnk")                # under a regular file: rank 0 fails ...
            raise AssertionError("save into a missing directory returned")
        except RuntimeError as e:                        # ... and every rank raises
            assert "rank 0" in str(e)
        with open(f"{tmp}/raised{rank}", "w") as f:
            f.write("1")
    finally:
        dist.destroy_process_group()


def test_save_world2_reports_rank0_failure_on_every_rank(tmp_path):
    """Advisor r4: with one writer, the other ranks must neither return before the checkpoint
    exists nor miss a failed write -- rank 0's outcome is broadcast."""
    mp.start_processes(_save_fail_worker, args=(str(tmp_path),), nprocs=2, start_method="spawn")
    assert (tmp_path / "raised0").exists() and (tmp_path / "raised1").exists()
