"""Inference paths: fp8 (OCP e4m3) FeatureNet-3D on the fp8 halo kernels."""
from .fp8 import Fp8FeatureNet3D, quantize_model

__all__ = ["Fp8FeatureNet3D", "quantize_model"]
