"""Public Python API: ``train()``, ``classify()``, ``evaluate()``, ``load()``,
``save()``, ``build_model()`` and ``search()``.

Reference parity: the de-facto entry point of the reference is the
``TensorflowGenerator(product, epochs, dataset, ...)`` constructor
(``tensorflow_generator.py:97-136``), which parses a product / template,
builds, trains, evaluates and scores robustness in one go.  Here the same
pipeline is split into composable calls:

    >>> import featurenet_amd as fn
    >>> res = fn.train("featurenet3d", data="voxel", epochs=2)        # 64^3, 24 classes
    >>> labels, probs = fn.classify(res.path, voxels)
    >>> res = fn.train("lenet5", data="mnist", epochs=12)              # NAS template
    >>> res = fn.train(product_tree, data="cifar", epochs=25)          # a PLEDGE product

``arch`` may be ``"featurenet3d"`` / a :class:`FeatureNet3DConfig`, an IR
:class:`ModelSpec`, a template name (``lenet5``, ``keras``, ...), or a product
tree (list of block dicts from :class:`~featurenet_amd.fm.products.ProductSet`).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from pathlib import Path

import numpy as np
import torch

from .ir.compile import CandidateNet, compile_model
from .ir.parse import parse_feature_model
from .ir.spec import ModelSpec
from .ir.templates import TEMPLATES
from .models.featurenet3d import FeatureNet3D, FeatureNet3DConfig, FeatureNet3DSeg
from .training.callbacks import reference_callbacks
from .training.checkpoint import read_checkpoint, save_checkpoint
from .training.data import Dataset, load_dataset
from .training.trainer import Trainer


@dataclass
class TrainResult:
    model: torch.nn.Module
    trainer: Trainer
    history: dict
    accuracy: float
    loss: float
    path: str | None = None
    spec: ModelSpec | None = None
    meta: dict = field(default_factory=dict)


def _is_featurenet3d(arch) -> bool:
    return isinstance(arch, FeatureNet3DConfig) or (isinstance(arch, str) and arch.lower() in
                                                     ("featurenet3d", "featurenet-3d", "featurenet"))


def build_model(arch, input_shape: tuple, num_classes: int, compat: bool = True, fill_defaults: bool = False):
    """-> (module, meta) where meta describes how to rebuild it from a checkpoint."""
    if _is_featurenet3d(arch):
        cfg = arch if isinstance(arch, FeatureNet3DConfig) else FeatureNet3DConfig(
            input_size=int(input_shape[0]), in_channels=int(input_shape[-1]), num_classes=num_classes)
        return FeatureNet3D(cfg), {"model_kind": "featurenet3d", "config": cfg.to_dict()}
    if isinstance(arch, str) and arch.lower() in ("featurenet3d-seg", "segmentation"):
        m = FeatureNet3DSeg(input_size=int(input_shape[0]), in_channels=int(input_shape[-1]), num_classes=num_classes)
        return m, {"model_kind": "featurenet3d_seg", "input_size": int(input_shape[0]),
                   "in_channels": int(input_shape[-1]), "num_classes": num_classes}
    if isinstance(arch, ModelSpec):
        spec = arch
    elif isinstance(arch, str):
        if arch not in TEMPLATES:
            raise ValueError(f"unknown architecture / template {arch!r}")
        spec = parse_feature_model(arch, name=arch)
    else:
        spec = parse_feature_model(arch)
    net = compile_model(spec, tuple(input_shape), num_classes, compat=compat, fill_defaults=fill_defaults)
    spec.nb_params, spec.nb_layers, spec.nb_flops = net.nb_params, net.nb_layers, net.flops_per_sample
    return net, {"model_kind": "candidate", "spec": spec.to_dict(), "input_shape": list(input_shape),
                 "num_classes": num_classes, "compat": compat, "fill_defaults": fill_defaults}


def _resolve_data(data, batch_size) -> Dataset:
    if isinstance(data, Dataset):
        return data
    if isinstance(data, str):
        return load_dataset(data)
    if isinstance(data, (tuple, list)) and len(data) == 4:
        xtr, ytr, xte, yte = data
        ncls = int(max(np.max(ytr), np.max(yte)) + 1)
        return Dataset("custom", xtr, ytr, xte, yte, ncls, tuple(np.asarray(xtr).shape[1:]))
    raise ValueError("data must be a dataset name, a Dataset or (x_train, y_train, x_test, y_test)")


def train(arch="featurenet3d", data="voxel", epochs: int = 12, batch_size: int = 128, lr: float = 1e-3,
          optimizer: str = "adam", device=None, callbacks=None, augment: bool = False, scheduler: bool = False,
          save_path: str | None = None, compat: bool = True, fill_defaults: bool = False, verbose: int = 1,
          seed: int = 0, robustness: list | None = None, graph: bool = True, precise_bn: int = 32) -> TrainResult:
    """Build + train + evaluate one architecture (the reference ``TensorflowGenerator`` pipeline)."""
    torch.manual_seed(seed)
    ds = _resolve_data(data, batch_size)
    model, meta = build_model(arch, ds.input_shape, ds.num_classes, compat=compat, fill_defaults=fill_defaults)
    meta.update({"dataset": ds.name, "synthetic_data": ds.synthetic})
    trainer = Trainer(model, optimizer=optimizer, lr=lr, device=device, meta=meta, graph=graph, precise_bn=precise_bn)
    cbs = list(callbacks) if callbacks is not None else reference_callbacks(scheduler)
    packed = ds.input_shape[0] if ds.packed else None
    hist = trainer.fit(ds.x_train, ds.y_train, epochs=epochs, batch_size=batch_size,
                       validation_data=(ds.x_test, ds.y_test), callbacks=cbs, augment=augment,
                       packed_size=packed, verbose=verbose, seed=seed)
    loss, acc = trainer.evaluate(ds.x_test, ds.y_test, packed_size=packed)
    meta.update({"accuracy": acc, "test_loss": loss})
    trainer.meta.update(meta)
    spec = None
    if meta["model_kind"] == "candidate":
        spec = ModelSpec.from_dict(meta["spec"])
        spec.accuracy, spec.status, spec.history = acc, "trained", hist.history
    if robustness:
        from .robust.evaluate import eval_robustness

        scores = eval_robustness(model, ds, robustness, device=trainer.device)
        meta["robustness"] = scores
        if spec is not None:
            spec.robustness_score = scores.get("score", 0.0)
    path = None
    if save_path:
        path = str(trainer.save(save_path))
    return TrainResult(model, trainer, hist.history, acc, loss, path, spec, meta)


def save(model: torch.nn.Module, path: str | Path, meta: dict) -> Path:
    return save_checkpoint(path, model, meta)


def load(path: str | Path, device=None) -> tuple[torch.nn.Module, dict]:
    """Rebuild a model from a ``.fnk`` checkpoint (weights + architecture)."""
    meta, state, _ = read_checkpoint(path)
    kind = meta.get("model_kind")
    if kind == "featurenet3d":
        model = FeatureNet3D(FeatureNet3DConfig.from_dict(meta["config"]))
    elif kind == "featurenet3d_seg":
        model = FeatureNet3DSeg(meta["input_size"], meta["in_channels"], meta["num_classes"])
    elif kind == "candidate":
        spec = ModelSpec.from_dict(meta["spec"])
        model = compile_model(spec, tuple(meta["input_shape"]), int(meta["num_classes"]),
                              compat=meta.get("compat", True), fill_defaults=meta.get("fill_defaults", False))
    else:
        raise ValueError(f"{path}: unknown model kind {kind!r}")
    model.load_state_dict(state)
    if device is None:
        device = "cuda" if torch.cuda.is_available() else "cpu"
    return model.to(device).eval(), meta


@torch.no_grad()
def classify(model, x, batch_size: int = 256, device=None, packed_size: int | None = None, fp8_calib=None):
    """Predict classes for ``x`` -> (labels int64 [N], probabilities [N, C]).

    ``model`` may be a module or a checkpoint path.  For voxel models ``x`` is
    ``[N, S, S, S]`` / ``[N, S, S, S, 1]`` occupancy (any dtype) or bit-packed
    ``uint8 [N, S^3/8]`` with ``packed_size=S``.

    ``fp8_calib`` (FeatureNet-3D on the GPU): calibration voxels in the same format as ``x``; the
    model then runs in fp8 (OCP e4m3) with the numerics its calibration check chooses --
    block-scaled activations, per-tensor scales, or bf16 when neither agrees with the bf16 model
    on >= 99 % of the calibration set (``inference.fp8.quantize_model(fallback=True)``,
    profiles/r6_fp8_fallback.md).
    """
    if isinstance(model, (str, Path)):
        model, _ = load(model, device)
    dev = next(model.parameters()).device
    model.eval()
    from .training.data import unpack_voxels

    def prep(xb):
        xb = xb.to(dev)
        if packed_size is not None:
            xb = unpack_voxels(xb, packed_size)
        return xb.to(torch.bfloat16) if dev.type == "cuda" else xb.float()

    fwd = model
    if fp8_calib is not None:
        from .models.featurenet3d import FeatureNet3D

        if dev.type != "cuda" or not isinstance(model, FeatureNet3D):
            raise ValueError("fp8 inference (fp8_calib) takes a FeatureNet-3D model on the GPU")
        from .inference.fp8 import quantize_model

        ct = torch.as_tensor(np.asarray(fp8_calib)) if not isinstance(fp8_calib, torch.Tensor) else fp8_calib
        fwd = quantize_model(model, prep(ct), fallback=True)
    xt = torch.as_tensor(np.asarray(x)) if not isinstance(x, torch.Tensor) else x
    probs = []
    for i in range(0, len(xt), batch_size):
        probs.append(torch.softmax(fwd(prep(xt[i:i + batch_size])).float(), -1).cpu())
    p = torch.cat(probs).numpy() if probs else np.zeros((0, 0), np.float32)
    return p.argmax(-1), p


def evaluate(model, x, y, batch_size: int = 256, packed_size: int | None = None) -> float:
    labels, _ = classify(model, x, batch_size, packed_size=packed_size)
    return float((labels == np.asarray(y)).mean())


def search(**kwargs):
    """Run the mutation-driven NAS (reference ``FullEvolution.run``); see
    :func:`featurenet_amd.search.evolution.run_evolution` for arguments."""
    from .search.evolution import run_evolution

    return run_evolution(**kwargs)
