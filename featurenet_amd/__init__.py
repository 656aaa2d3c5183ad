"""featurenet_amd -- a MI355X-native (gfx950 / CDNA4) FeatureNet framework.

Feature-model driven neural architecture search (sampling, mutation,
evolution, robustness scoring) plus the FeatureNet-3D voxel workload, on
hand-written HIP/MFMA kernels, RCCL data parallelism and a native C++ runtime.
"""
__version__ = "0.1.0"
