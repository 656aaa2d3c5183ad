"""featurenet_amd -- a MI355X-native (gfx950 / CDNA4) FeatureNet framework.

Feature-model driven neural architecture search (sampling, mutation,
evolution, robustness scoring) plus the FeatureNet-3D voxel workload, on
hand-written HIP/MFMA kernels, RCCL data parallelism and a native C++ runtime.
"""
__version__ = "0.1.0"

# Public API (``featurenet_amd.api``), resolved lazily so importing the package
# stays cheap and does not pull in torch-heavy modules until they are used.
_API = ("train", "classify", "evaluate", "load", "save", "build_model", "search", "TrainResult")


def __getattr__(name):
    if name in _API:
        from . import api

        return getattr(api, name)
    raise AttributeError(f"module 'featurenet_amd' has no attribute {name!r}")


__all__ = list(_API)
