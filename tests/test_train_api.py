"""Trainer, callbacks, checkpoint format and the public train/classify API (CPU path)."""
import math

import numpy as np
import pytest
import torch

import featurenet_amd as fn
from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig
from featurenet_amd.training import callbacks as C
from featurenet_amd.training.checkpoint import FORMAT, read_checkpoint
from featurenet_amd.training.trainer import Trainer


def _images(n, seed=0):
    rng = np.random.default_rng(seed)
    y = rng.integers(0, 2, n)
    x = rng.random((n, 28, 28, 1)).astype(np.float32) * 0.2
    x[y == 1, :14] += 0.8          # learnable: bright top half = class 1
    return x, y


def _voxels(n, size=16, seed=0):
    rng = np.random.default_rng(seed)
    y = rng.integers(0, 2, n)
    x = (rng.random((n, size, size, size, 1)) < 0.05).astype(np.float32)
    x[y == 1, : size // 2, : size // 2, : size // 2] = 1.0   # a solid corner block = class 1
    return x, y


def test_api_train_save_load_classify(tmp_path):
    xtr, ytr = _images(256, 0)
    xte, yte = _images(64, 1)
    res = fn.train("lenet5", data=(xtr, ytr, xte, yte), epochs=3, batch_size=32, verbose=0,
                   save_path=str(tmp_path / "lenet.fnk"))
    assert res.accuracy > 0.9
    assert res.spec is not None and res.spec.status == "trained"
    labels, probs = fn.classify(res.path, xte, device="cpu")
    assert probs.shape == (64, 2)
    np.testing.assert_allclose(probs.sum(1), 1.0, rtol=1e-5)
    assert (labels == yte).mean() == pytest.approx(res.accuracy, abs=1e-6)
    model, meta = fn.load(res.path, device="cpu")
    assert meta["model_kind"] == "candidate" and meta["format"] == FORMAT
    assert fn.evaluate(model, xte, yte) == pytest.approx(res.accuracy, abs=1e-6)


def test_classify_fp8_needs_featurenet3d_on_gpu():
    """classify(fp8_calib=...) is the GPU fp8 path of FeatureNet-3D: refused on the CPU."""
    m = FeatureNet3D(FeatureNet3DConfig.tiny())
    x, _ = _voxels(4, 16, 0)
    labels, probs = fn.classify(m, x, device="cpu")
    assert probs.shape[0] == 4
    with pytest.raises(ValueError, match="fp8"):
        fn.classify(m, x, device="cpu", fp8_calib=x)


def test_featurenet3d_tiny_learns_on_cpu():
    """BASELINE config 1: 16^3-voxel 2-class tiny 3D-CNN on the CPU reference path."""
    xtr, ytr = _voxels(128, 16, 0)
    xte, yte = _voxels(64, 16, 1)
    res = fn.train(FeatureNet3DConfig.tiny(), data=(xtr, ytr, xte, yte), epochs=4, batch_size=16, verbose=0)
    assert res.accuracy >= 0.9
    assert all(math.isfinite(v) for v in res.history["loss"])


def test_checkpoint_roundtrip_with_optimizer(tmp_path):
    torch.manual_seed(0)
    m = FeatureNet3D(FeatureNet3DConfig.tiny())
    tr = Trainer(m, lr=1e-3, device="cpu", meta={"model_kind": "featurenet3d",
                                                  "config": FeatureNet3DConfig.tiny().to_dict()})
    x, y = _voxels(8)
    tr.train_step(torch.as_tensor(x), torch.as_tensor(y))
    p = tr.save(tmp_path / "m.fnk")
    meta, state, opt = read_checkpoint(p)
    assert meta["format"] == FORMAT
    for k, v in m.state_dict().items():
        assert torch.equal(state[k], v.cpu())
    assert opt and any(torch.is_tensor(v) and v.abs().sum() > 0 for v in opt.values())
    m2, _ = fn.load(p, device="cpu")
    with torch.no_grad():
        torch.testing.assert_close(m2(torch.as_tensor(x)), m.eval()(torch.as_tensor(x)))


class _FakeTrainer:
    def __init__(self, lr=1e-3):
        self.lr, self.stop_training = lr, False
        self.model = torch.nn.Linear(2, 2)

    def get_lr(self):
        return self.lr

    def set_lr(self, v):
        self.lr = v


def test_reference_lr_schedule():
    assert C.reference_lr_schedule(0) == 1e-3
    assert C.reference_lr_schedule(81) == pytest.approx(1e-4)
    assert C.reference_lr_schedule(121) == pytest.approx(1e-5)
    assert C.reference_lr_schedule(161) == pytest.approx(1e-6)
    assert C.reference_lr_schedule(181) == pytest.approx(0.5e-6)


def test_reduce_lr_on_plateau_and_early_stopping():
    t = _FakeTrainer()
    r = C.ReduceLROnPlateau(patience=2)
    for e, v in enumerate([1.0, 1.0, 1.0]):
        r.on_epoch_end(t, e, {"val_loss": v})
    assert t.lr == pytest.approx(1e-3 * math.sqrt(0.1))
    es = C.EarlyStopping(patience=2)
    for e, v in enumerate([0.5, 0.505, 0.509]):
        es.on_epoch_end(t, e, {"val_acc": v})
    assert t.stop_training and es.stopped_epoch == 2


def test_model_checkpoint_restores_best():
    t = _FakeTrainer()
    mc = C.ModelCheckpoint()
    mc.on_epoch_end(t, 0, {"val_loss": 0.5})
    best = {k: v.clone() for k, v in t.model.state_dict().items()}
    with torch.no_grad():
        t.model.weight.add_(1.0)
    mc.on_epoch_end(t, 1, {"val_loss": 0.9})
    mc.on_train_end(t)
    assert torch.equal(t.model.weight, best["weight"])


def test_sgdr_cosine():
    t = _FakeTrainer()
    s = C.SGDRScheduler(min_lr=0.0, max_lr=1.0, steps_per_epoch=2, cycle_length=1)
    s.on_train_begin(t)
    s.on_batch_end(t, 0, {})
    assert t.lr == pytest.approx(0.5)
    s.on_batch_end(t, 1, {})
    assert t.lr == pytest.approx(0.0, abs=1e-12)
    s.on_epoch_end(t, 0, {})
    assert s.batch_since_restart == 0 and s.cycle_length == 2


def test_segmentation_head_trains_per_voxel():
    """BASELINE config 4 (per-voxel segmentation head) on the CPU path: loss/accuracy are per voxel."""
    rng = np.random.default_rng(0)
    x = (rng.random((16, 16, 16, 16, 1)) < 0.3).astype(np.float32)
    y = np.zeros((16, 16, 16, 16), np.int64)
    y[:, :8] = 1                                   # lower half of every part is "feature"
    res = fn.train("segmentation", data=(x[:12], y[:12], x[12:], y[12:]), epochs=6, batch_size=4, lr=3e-3,
                   verbose=0)
    assert 0.0 <= res.accuracy <= 1.0
    assert res.accuracy > 0.9
    assert all(math.isfinite(v) for v in res.history["loss"])


def test_precise_bn_recalibration_is_batch_average():
    """PreciseBN: running stats become the plain average of the per-batch statistics."""
    from featurenet_amd.models.layers import BatchNorm, Dense
    from featurenet_amd.training.trainer import bn_modules

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.bn = BatchNorm(4, momentum=0.1)
            self.fc = Dense(4, 3)

        def forward(self, x):
            return self.fc(self.bn(x))

    torch.manual_seed(0)
    x = (torch.randn(32, 4) * torch.tensor([1.0, 2.0, 3.0, 4.0]) + torch.tensor([5.0, -1.0, 0.0, 2.0])).numpy()
    y = np.zeros(32, dtype=np.int64)
    tr = Trainer(Net(), device="cpu", precise_bn=4)
    assert [type(m).__name__ for m, _ in bn_modules(tr.model)] == ["BatchNorm"]
    n = tr.recalibrate_bn(x, y, batches=4, batch_size=8)
    assert n == 4
    assert tr.model.bn.momentum == 0.1                       # momentum restored
    xt = torch.from_numpy(x)
    torch.testing.assert_close(tr.model.bn.running_mean, xt.mean(0), rtol=1e-4, atol=1e-4)
    # average of unbiased per-batch variances (batches are a permutation of the data)
    perm_var = tr.model.bn.running_var
    assert torch.all(perm_var > 0.5 * xt.var(0)) and torch.all(perm_var < 1.5 * xt.var(0))


def test_fit_recalibrates_before_validation():
    torch.manual_seed(0)
    from featurenet_amd.training.data import voxel_dataset

    ds = voxel_dataset(16, 8, size=32, num_classes=2, seed=3)
    model = FeatureNet3D(FeatureNet3DConfig(input_size=32, num_classes=2))
    tr = Trainer(model, device="cpu", precise_bn=2)
    calls = []
    orig = tr.recalibrate_bn
    tr.recalibrate_bn = lambda *a, **k: calls.append(1) or orig(*a, **k)
    tr.fit(ds.x_train, ds.y_train, epochs=2, batch_size=8, validation_data=(ds.x_test, ds.y_test),
           packed_size=32, verbose=0)
    assert len(calls) == 2 and tr._bn_fresh


def test_resume_from_checkpoint_is_bit_identical(tmp_path):
    """Checkpoint at an epoch end = weights + Adam moments/step + every random generator
    (torch, numpy, python, the loader's shuffle generator).  A fresh trainer resumed from it
    reproduces the remaining epochs' losses bit-for-bit (dropout masks and shuffle order
    included) -- SURVEY 5.4; reference best-checkpoint reload helpers.py:88-97,169-170."""
    import random

    import numpy as np
    import torch
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
            f = dropout(f, 0.3, self.training)          # torch's CPU generator on the CPU path
            return self.body.fc2(self.body.fc1(f), out_fp32=True)

    rs = np.random.RandomState(0)
    x = (rs.rand(48, 16, 16, 16) < 0.3).astype(np.float32)
    y = rs.randint(0, 2, 48).astype(np.int64)

    class SaveAt(Callback):
        def on_epoch_end(self, trainer, epoch, logs):
            if epoch == 1:
                trainer.save(tmp_path / "mid.fnk")

    torch.manual_seed(0)
    tr = Trainer(Net(), device="cpu", precise_bn=0)
    h = tr.fit(x, y, epochs=4, batch_size=8, callbacks=[SaveAt()], verbose=0, seed=3)
    full = h.history["loss"]

    torch.manual_seed(123)                              # different init: everything must come from the file
    random.seed(99)
    np.random.seed(7)
    tr2 = Trainer(Net(), device="cpu", precise_bn=0)
    done = tr2.resume(tmp_path / "mid.fnk")
    assert done == 2 and tr2.opt.t == tr.opt.t // 2
    h2 = tr2.fit(x, y, epochs=4, batch_size=8, verbose=0, seed=3, initial_epoch=done)
    assert h2.history["loss"][:2] == full[:2]          # the history came back with the weights
    assert h2.history["loss"][2:] == full[2:], (h2.history["loss"], full)
    for a, b in zip(tr.model.parameters(), tr2.model.parameters()):
        assert torch.equal(a, b)


def test_epoch_metrics_accumulate_like_the_per_step_reductions():
    """Trainer's device-side epoch sums (one add per step) equal the reference per-step sums,
    including a smaller last batch and per-voxel correct maps (the scalar fallback)."""
    import torch

    from featurenet_amd.training.trainer import _EpochMetrics

    torch.manual_seed(0)
    m = _EpochMetrics(torch.device("cpu"))
    ref_loss, ref_corr = 0.0, 0
    for n in (64, 64, 17):
        loss = torch.rand(())
        corr = torch.randint(0, 2, (n,), dtype=torch.int32)
        m.add(loss, corr, n)
        ref_loss += float(loss) * n
        ref_corr += int(corr.sum())
    big = torch.randint(0, 2, (70000,), dtype=torch.int32)        # per-voxel: beyond the vector size
    m.add(torch.tensor(0.5), big, big.numel())
    ref_loss += 0.5 * big.numel()
    ref_corr += int(big.sum())
    ls, cs = m.totals()
    assert abs(float(ls) - ref_loss) < 1e-6 * ref_loss
    assert int(cs) == ref_corr
