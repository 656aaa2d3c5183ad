"""Robustness evaluation policy of a trained candidate.

Reference: ``TensorflowGenerator.eval_robustness`` / ``eval_attack_robustness``
(``tensorflow_generator.py:151-218``):

* skipped when the model's accuracy is below 0.5;
* norm 2 everywhere; CLEVER with radius 2, nb_batches 10, batch 5,
  pool_factor 3, averaged over the robustness set;
* attacks on the first ``robustness_set_size`` test samples (500 by default);
  PGD eps 1 / step 0.1; CW untargeted;
* per attack the score is the tuple (mean relative perturbation, clean
  accuracy, adversarial accuracy);
* the model's ``robustness_score`` is the first requested metric's first
  element (CLEVER's average when CLEVER is requested first);
* clip values (0, 255) as in the reference although data lives in [0, 1]
  (kept as the default; pass ``clip=(0, 1)`` for the tight box).

Errors inside an attack are caught and reported, never propagated (the
reference swallows them too).
"""
from __future__ import annotations

import time
import traceback

import numpy as np
import torch

from . import attacks as A
from .metrics import clever_u_batch, empirical_robustness

ATTACK_PARAMS = {"pgd": {"eps": 1.0, "eps_step": 0.1}, "cw": {}, "fgsm": {}}


def _as_tensor(x, device) -> torch.Tensor:
    t = torch.as_tensor(np.asarray(x)) if not isinstance(x, torch.Tensor) else x
    return t.to(device).float()


def eval_attack_robustness(model, x, y, attack: str, norm=2, clip=(0.0, 255.0)) -> tuple[float, float, float]:
    params = dict(ATTACK_PARAMS.get(attack, {}))
    params["norm"] = norm
    if attack != "cw":
        params["clip"] = clip
    else:
        params["clip"] = clip
    score, adv = empirical_robustness(model, x, attack, params)
    y = y.to(x.device)
    clean = float((A.predict(model, x).argmax(-1) == y).float().mean())
    advacc = float((A.predict(model, adv).argmax(-1) == y).float().mean())
    return float(score), clean, advacc


def eval_robustness(model, dataset, metrics=("clever", "pgd", "cw", "fgsm"), set_size: int = 500, device=None,
                    accuracy: float | None = None, norm=2, clip=(0.0, 255.0), clever_samples: int | None = None,
                    packed_size: int | None = None) -> dict:
    """Score ``model`` on ``dataset`` (a :class:`Dataset` or an ``(x, y)`` pair)."""
    if accuracy is not None and accuracy < 0.5:
        return {"skipped": "accuracy < 0.5", "score": 0.0}
    if device is None:
        device = next(model.parameters()).device
    if isinstance(dataset, tuple):
        xs, ys = dataset
    else:
        xs, ys = dataset.robustness_set(set_size)
        if getattr(dataset, "packed", False):
            packed_size = dataset.input_shape[0]
    x = torch.as_tensor(np.asarray(xs)).to(device) if not isinstance(xs, torch.Tensor) else xs.to(device)
    if packed_size is not None:
        from ..training.data import unpack_voxels

        x = unpack_voxels(x, packed_size)
    x = x.float()[:set_size]
    y = torch.as_tensor(np.asarray(ys)).long().to(device)[:set_size]
    model.eval()
    t0 = time.time()
    out: dict = {}
    for m in metrics:
        try:
            if m == "clever":
                n = len(x) if clever_samples is None else min(clever_samples, len(x))
                # every sample at once: batched class-gradient passes over all pools, one batched
                # reverse-Weibull fit (the reference's per-sample loop, same draws)
                scores = clever_u_batch(model, x[:n], nb_batches=10, batch_size=5, radius=2 if norm == 2 else 0.1,
                                        norm=norm, pool_factor=3, clip=clip) if n else []
                out["clever"] = float(np.mean(scores)) if len(scores) else 0.0
            else:
                out[m] = eval_attack_robustness(model, x, y, m, norm, clip)
        except Exception as e:  # reference: errors are printed and swallowed
            out[m] = None
            out.setdefault("errors", {})[m] = f"{type(e).__name__}: {e}\n{traceback.format_exc(limit=3)}"
    first = metrics[0] if metrics else None
    v = out.get(first)
    out["score"] = float(v[0]) if isinstance(v, tuple) else (float(v) if isinstance(v, float) else 0.0)
    out["time_s"] = time.time() - t0
    model.train()
    return out
