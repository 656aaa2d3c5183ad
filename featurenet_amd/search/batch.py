"""Batch product trainers, product (re)trainer and checkpoint retrainer.

* :func:`train_product_set` -- reference ``full.py`` / ``full_mnist.py`` /
  ``full_cifar.py`` (``full.py:8-38``): for every product of a ``.pdt`` (index
  window / filter), dump the product tree JSON, train it on each dataset and
  append one report line per dataset (``"\\r\\n{i}: {acc} {stop} {time} {params}
  {flops} {acc#..|val_acc#..}"``).  Trials go through the
  :class:`~featurenet_amd.search.trial.TrialScheduler`, so an 8-GPU node
  trains 8 products at once (the reference is strictly serial).
* :func:`train_from_product` / :func:`train_from_json` -- reference
  ``pledge_trainer.py:11-71``: retrain a product by index from a binary
  ``.pdt``, or a slice of an exported vector list, and export the resulting
  :class:`KerasFeatureVector` list.
* :func:`retrain_checkpoint` -- reference ``utils/retrainer.py``: reload a saved
  model and continue training.
"""
from __future__ import annotations

import json
from pathlib import Path

from ..fm.products import ProductSet
from ..ir.parse import parse_feature_model
from ..utils.reports import KerasFeatureVector, report_line, spec_vector
from .trial import TrialConfig, TrialScheduler


def _history_field(spec) -> dict:
    h = spec.history or {}
    return {k: list(h.get(k, [])) for k in ("acc", "val_acc")}


def train_product_set(target: str, datasets=("mnist",), epochs: int = 12, min_index: int = 0, max_index: int = 0,
                      filter_indices=(), output_folder: str = "./products/", scheduler: TrialScheduler | None = None,
                      cfg: TrialConfig | None = None, depth: int = 1) -> list:
    """``target`` is the product file path without ``.pdt`` (as in the reference)."""
    pdt = target if target.endswith(".pdt") else target + ".pdt"
    stem = target[:-4] if target.endswith(".pdt") else target
    ps = ProductSet(pdt)
    Path(output_folder).mkdir(parents=True, exist_ok=True)
    scheduler = scheduler or TrialScheduler()
    todo = []
    for index, (product, features) in enumerate(ps.format_products()):
        if index >= min_index and (not filter_indices or index in filter_indices):
            Path(output_folder, f"{Path(stem).name}_{index}.json").write_text(json.dumps(product))
            spec = parse_feature_model(product, name=f"{Path(stem).name}_{index}", depth=depth,
                                       product_features=sorted(features, key=lambda k: abs(int(k))))
            todo.append((index, spec))
        if max_index and index == max_index:
            break
    results = []
    for ds in datasets:
        c = TrialConfig(**{**(cfg.to_dict() if cfg else {}), "dataset": ds, "epochs": epochs})
        trained = scheduler.map([s for _, s in todo], c)
        log = f"{stem}_{ds}_{epochs}epochs_{depth}.txt"
        with open(log, "a") as f:
            for (index, _), s in zip(todo, trained):
                tt = next((m.get("trial_time_s") for m in s.metrics if isinstance(m, dict) and "trial_time_s" in m), 0)
                f.write(report_line(index, s.accuracy, False, tt, s.nb_params, s.nb_flops, _history_field(s)))
        results.append((ds, trained))
    return results


def _spec_from_bits(ps: ProductSet, bits, name: str):
    parsed = ps.format_product(original_product=[1 if b else 0 for b in bits])
    if not parsed:
        return None
    tree, _ = parsed
    s = parse_feature_model(tree, name=name)
    s.features = [1 if b else 0 for b in bits]
    return s


def train_from_product(pdt: str, index: int, export_file: str = "", epochs: int = 5, batch_size: int = 64,
                       dataset: str = "mnist", scheduler: TrialScheduler | None = None, cfg: TrialConfig | None = None):
    ps = ProductSet(pdt, binary_products=True)
    spec = _spec_from_bits(ps, ps.products[int(index)], f"p{int(index)}")
    c = TrialConfig(**{**(cfg.to_dict() if cfg else {}), "dataset": dataset, "epochs": epochs,
                       "batch_size": batch_size or 64})
    out = (scheduler or TrialScheduler()).map([spec], c)[0]
    vec = spec_vector(out)
    if export_file:
        Path(export_file).write_text(json.dumps([vec.to_vector()]))
    return vec


def train_from_json(pdt: str, products_file: str, index=None, export_file: str = "", epochs: int = 5,
                    batch_size: int = 64, dataset: str = "mnist", scheduler: TrialScheduler | None = None,
                    cfg: TrialConfig | None = None) -> list:
    """``index``: None (all), ``[i]`` (one) or ``[a, b]`` (slice), as ``-i a-b`` in the reference."""
    ps = ProductSet(pdt, binary_products=True)
    vecs = [KerasFeatureVector.from_vector(v) for v in json.loads(Path(products_file).read_text())]
    if index is not None:
        idx = [int(i) for i in index]
        vecs = [vecs[idx[0]]] if len(idx) == 1 else vecs[max(0, idx[0]):min(len(vecs), idx[1])]
    specs = [s for s in (_spec_from_bits(ps, v.features, v.name or f"v{i}") for i, v in enumerate(vecs)) if s]
    c = TrialConfig(**{**(cfg.to_dict() if cfg else {}), "dataset": dataset, "epochs": epochs,
                       "batch_size": batch_size or 64})
    out = [spec_vector(s) for s in (scheduler or TrialScheduler()).map(specs, c)]
    for old, new in zip(vecs, out):
        print(f"original accuracy {old.accuracy} new accuracy {new.accuracy}")
    if export_file:
        Path(export_file).write_text(json.dumps([v.to_vector() for v in out]))
    return out


def retrain_checkpoint(model_path: str, epochs: int = 100, dataset: str = "cifar", augment: bool = True,
                       batch_size: int = 64, save_path: str | None = None, device=None, verbose: int = 1):
    """Reload a ``.fnk`` checkpoint (weights + optimizer state) and continue training."""
    from ..api import load
    from ..training.callbacks import reference_callbacks
    from ..training.checkpoint import read_checkpoint
    from ..training.data import load_dataset
    from ..training.trainer import Trainer

    model, meta = load(model_path, device=device)
    _, _, opt_state = read_checkpoint(model_path)
    ds = load_dataset(dataset)
    ometa = meta.get("optimizer") or {}
    tr = Trainer(model, optimizer=meta.get("optimizer_name", "adam"), lr=float(ometa.get("lr", 1e-3)),
                 device=next(model.parameters()).device, meta=meta)
    if opt_state:   # resume the optimizer moments and step count
        tr.opt.load_state_dict({**ometa, **{k: v.to(tr.device) for k, v in opt_state.items()}})
    packed = ds.input_shape[0] if ds.packed else None
    tr.fit(ds.x_train, ds.y_train, epochs=epochs, batch_size=batch_size, validation_data=(ds.x_test, ds.y_test),
           callbacks=reference_callbacks(True), augment=augment, packed_size=packed, verbose=verbose)
    loss, acc = tr.evaluate(ds.x_test, ds.y_test, packed_size=packed)
    tr.meta.update({"accuracy": acc, "test_loss": loss})
    if save_path:
        tr.save(save_path)
    return acc, tr
