"""The stock-PyTorch convergence oracle of ``bench/accuracy.py --impl torch`` is the same network as
the native FeatureNet-3D: built from the native model's tensors (conv weights converted from
[K, KD, KH, KW, C], channels-last flatten before FC1), its forward must equal the native model's
CPU (fp32 reference-op) forward, in training mode (batch statistics) and in eval mode."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def test_oracle_matches_native_cpu_forward():
    from bench.accuracy import OracleFeatureNet3D
    from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig

    torch.manual_seed(0)
    native = FeatureNet3D(FeatureNet3DConfig(input_size=32, num_classes=5))
    oracle = OracleFeatureNet3D(native)
    x = (torch.rand(3, 32, 32, 32, 1) < 0.3).float()
    for train in (True, False):
        native.train(train)
        oracle.train(train)
        a, b = native(x).float(), oracle(x)
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-4), (train, (a - b).abs().max())
    # the running statistics moved the same way in the training-mode forward
    for i, c in enumerate(native.convs):
        assert torch.allclose(c.running_mean, getattr(oracle, f"rm{i}"), rtol=1e-4, atol=1e-5)
