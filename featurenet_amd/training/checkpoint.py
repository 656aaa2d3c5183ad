"""Checkpoint format: one ``.fnk`` file = safetensors blobs + JSON header.

Reference: Keras HDF5 ``.h5`` full-model files (``tensorflow_generator.py:255,
265-268``, ``helpers.py:88-97,169-170``), reloaded by ``utils/retrainer.py``.
The new format is stable and self-describing:

* tensors: ``model.*`` (state dict, fp32 masters + BN running stats),
  optionally ``optim.*`` (optimizer moments) and ``rng.*`` (generator states:
  torch CPU, every CUDA device, the data loader's shuffle/augment generator;
  numpy's and Python's global states go into the JSON header), so that a
  resumed run continues bit-for-bit;
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


def capture_rng(generators: dict | None = None) -> tuple[dict, dict]:
    """(tensors, json) snapshot of every random state a training run draws from: torch's CPU
    generator, each CUDA device's default generator, the named extra generators (e.g. the
    data loader's), numpy's and Python's global generators."""
    import random

    import numpy as np

    tensors = {"rng.torch_cpu": torch.get_rng_state()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        for i, st in enumerate(torch.cuda.get_rng_state_all()):
            tensors[f"rng.cuda.{i}"] = st
    for name, g in (generators or {}).items():
        if g is not None:
            tensors[f"rng.gen.{name}"] = g.get_state()
    kind, keys, pos, has_gauss, cached = np.random.get_state()
    tensors["rng.numpy_keys"] = torch.from_numpy(np.asarray(keys, dtype=np.uint32).astype(np.int64))
    version, state, gauss = random.getstate()
    meta = {"numpy": [kind, int(pos), int(has_gauss), float(cached)],
            "python": [version, list(state), gauss]}
    return tensors, meta


def restore_rng(tensors: dict, meta: dict, generators: dict | None = None) -> None:
    """Inverse of :func:`capture_rng` (``tensors`` keyed without the ``rng.`` prefix)."""
    import random

    import numpy as np

    if "torch_cpu" in tensors:
        torch.set_rng_state(tensors["torch_cpu"].to(torch.uint8))
    cuda = sorted((int(k.split(".")[1]), v) for k, v in tensors.items() if k.startswith("cuda."))
    if cuda and torch.cuda.is_available():
        for i, st in cuda:
            if i < torch.cuda.device_count():
                torch.cuda.set_rng_state(st.to(torch.uint8), i)
    for name, g in (generators or {}).items():
        st = tensors.get(f"gen.{name}")
        if g is not None and st is not None:
            g.set_state(st.to(torch.uint8))
    if "numpy_keys" in tensors and meta.get("numpy"):
        kind, pos, has_gauss, cached = meta["numpy"]
        np.random.set_state((kind, tensors["numpy_keys"].numpy().astype(np.uint32), int(pos), int(has_gauss),
                             float(cached)))
    if meta.get("python"):
        version, state, gauss = meta["python"]
        random.setstate((version, tuple(state), gauss))


def save_checkpoint(path: str | Path, model: torch.nn.Module, meta: dict, optimizer=None,
                    rng: tuple[dict, dict] | None = None) -> Path:
    """``rng``: a :func:`capture_rng` snapshot to store with the weights."""
    path = Path(path)
    tensors = {f"model.{k}": v.detach().contiguous().cpu() for k, v in model.state_dict().items()}
    if rng is not None:
        for k, v in rng[0].items():
            tensors[k] = v.detach().contiguous().cpu()
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
    if rng is not None:
        header["rng"] = rng[1]
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


def read_rng(path: str | Path) -> tuple[dict, dict]:
    """The checkpoint's random-generator snapshot (tensors without the ``rng.`` prefix, json),
    empty when it has none."""
    meta, _, _ = read_checkpoint(path)
    from safetensors import safe_open

    out = {}
    with safe_open(str(path), framework="pt") as f:
        for k in f.keys():
            if k.startswith("rng."):
                out[k[len("rng."):]] = f.get_tensor(k)
    return out, meta.get("rng") or {}


def _jsonable(o):
    if isinstance(o, torch.Tensor):
        return o.tolist()
    if hasattr(o, "to_dict"):
        return o.to_dict()
    if isinstance(o, (set, tuple)):
        return list(o)
    return str(o)
