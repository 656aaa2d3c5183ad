"""End-to-end GPU paths beyond single kernels: input gradients through the native
stack (what the robustness attacks use), a NAS trial with robustness scoring,
and the hipGraph-captured trainer on the north-star model.

Reference parity: the attacks / CLEVER follow ``model/metrics.py`` and
``tensorflow_generator.py:151-218`` (ART is not importable here, so the checks
are the methods' defining properties, as in ``tests/test_robust.py``).
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from featurenet_amd import _native  # noqa: E402


def _native_loaded():
    assert _native.kernels_available(), "HIP kernel library (_C) must be built and loadable on the GPU box"


def test_input_gradient_matches_cpu_reference():
    """dL/dx of FeatureNet-3D (stride-2 stem dgrad + halo dgrads + BN/pool backward) vs the fp32 CPU path."""
    _native_loaded()
    from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig
    from featurenet_amd.robust.attacks import loss_gradient

    torch.manual_seed(0)
    cfg = FeatureNet3DConfig(input_size=32, num_classes=24, kernels=(5, 3, 3, 3), strides=(2, 1, 1, 1))
    m_cpu = FeatureNet3D(cfg).eval()
    m_gpu = FeatureNet3D(cfg)
    m_gpu.load_state_dict(m_cpu.state_dict())
    m_gpu = m_gpu.cuda().eval()
    x = (torch.rand(4, 32, 32, 32, 1) < 0.3).float()
    y = torch.randint(0, 24, (4,))
    g_cpu = loss_gradient(m_cpu, x, y)
    g_gpu = loss_gradient(m_gpu, x.cuda(), y.cuda()).float().cpu()
    assert torch.isfinite(g_gpu).all()
    cos = torch.nn.functional.cosine_similarity(g_gpu.flatten(), g_cpu.flatten(), dim=0).item()
    assert cos > 0.95, cos


def test_nas_trial_with_robustness_on_gpu():
    """One reference-style candidate (lenet5 template) trained on GPU, then FGSM / PGD / CW / CLEVER scored."""
    _native_loaded()
    from featurenet_amd.ir.parse import parse_feature_model
    from featurenet_amd.search.trial import TrialConfig, run_trial

    spec = parse_feature_model("lenet5", name="lenet5_gpu")
    cfg = TrialConfig(dataset="mnist", epochs=3, batch_size=64, attacks=["fgsm", "pgd", "cw", "clever"],
                      robustness_set_size=24, clever_samples=2, synthetic_sizes=(3000, 600), seed=1)
    out = run_trial(spec, cfg, device="cuda")
    assert out.status == "trained", out.error
    assert out.accuracy > 0.5
    for k in ("fgsm", "pgd", "cw"):
        v = getattr(out, f"{k}_score")
        assert v is not None and all(math.isfinite(float(t)) for t in v), (k, v)
        assert float(v[2]) <= float(v[1]) + 1e-6, (k, v)     # adversarial acc <= clean acc
    assert out.clever_score is not None and math.isfinite(out.clever_score) and out.clever_score >= 0


def test_graph_trainer_featurenet3d_learns():
    """hipGraph-captured FeatureNet-3D steps on the procedural voxel set: loss falls, eval agrees with classify()."""
    _native_loaded()
    import featurenet_amd as fn
    from featurenet_amd.training.data import voxel_dataset

    ds = voxel_dataset(24 * 24, 24 * 4, size=32, num_classes=24, seed=5)
    res = fn.train("featurenet3d", data=ds, epochs=4, batch_size=32, verbose=0, callbacks=[], graph=True)
    assert res.trainer.graph_mode
    losses = res.history["loss"]
    assert losses[-1] < losses[0] * 0.8, losses
    labels, probs = fn.classify(res.model, ds.x_test, packed_size=32)
    assert probs.shape == (len(ds.y_test), 24)
    assert abs(float((labels == np.asarray(ds.y_test)).mean()) - res.accuracy) < 1e-6
