"""Checkpoint format: one ``.fnk`` file = safetensors blobs + JSON header.

Reference: Keras HDF5 ``.h5`` full-model files (``tensorflow_generator.py:255,
265-268``, ``helpers.py:88-97,169-170``), reloaded by ``utils/retrainer.py``.
The new format is stable and self-describing:

* tensors: ``model.*`` (state dict, fp32 masters + BN running stats) and
  optionally ``optim.*`` (optimizer moments);
* metadata (safetensors string header, key ``featurenet``): format version,
  model kind (``featurenet3d`` | ``candidate``), the architecture (FeatureNet3D
  config or the IR :class:`ModelSpec` JSON with its product bit vector), input
  shape, number of classes, optimizer scalars, metrics/history and free-form
  user fields.

Loading never executes code from the file (safetensors + JSON only).
"""
from __future__ import annotations

import json
from pathlib import Path

import torch
from safetensors.torch import load_file, save_file

FORMAT = "featurenet_amd/1"


def save_checkpoint(path: str | Path, model: torch.nn.Module, meta: dict, optimizer=None) -> Path:
    path = Path(path)
    tensors = {f"model.{k}": v.detach().contiguous().cpu() for k, v in model.state_dict().items()}
    opt_meta = None
    if optimizer is not None:
        sd = optimizer.state_dict()
        opt_meta = {}
        for k, v in sd.items():
            if isinstance(v, torch.Tensor):
                tensors[f"optim.{k}"] = v.detach().contiguous().cpu()
            else:
                opt_meta[k] = v
    header = dict(meta)
    header["format"] = FORMAT
    if opt_meta is not None:
        header["optimizer"] = opt_meta
    path.parent.mkdir(parents=True, exist_ok=True)
    tmp = path.with_suffix(path.suffix + ".tmp")
    save_file(tensors, str(tmp), metadata={"featurenet": json.dumps(header, default=_jsonable)})
    tmp.replace(path)   # atomic publish
    return path


def read_checkpoint(path: str | Path) -> tuple[dict, dict, dict]:
    """-> (meta, model_state, optim_tensors)."""
    from safetensors import safe_open

    path = str(path)
    with safe_open(path, framework="pt") as f:
        md = f.metadata() or {}
    meta = json.loads(md.get("featurenet", "{}"))
    if meta.get("format") != FORMAT:
        raise ValueError(f"{path}: not a {FORMAT} checkpoint")
    tensors = load_file(path)
    model = {k[len("model."):]: v for k, v in tensors.items() if k.startswith("model.")}
    optim = {k[len("optim."):]: v for k, v in tensors.items() if k.startswith("optim.")}
    return meta, model, optim


def _jsonable(o):
    if isinstance(o, torch.Tensor):
        return o.tolist()
    if hasattr(o, "to_dict"):
        return o.to_dict()
    if isinstance(o, (set, tuple)):
        return list(o)
    return str(o)
