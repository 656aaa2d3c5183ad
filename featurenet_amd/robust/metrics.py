"""Robustness metrics: empirical robustness, loss sensitivity and CLEVER.

Reference: the vendored ART metrics module ``model/metrics.py:57-324``
(``empirical_robustness``, ``loss_sensitivity``, ``clever``, ``clever_u``,
``clever_t``).  Gradients are computed in batches on the GPU
(:func:`featurenet_amd.robust.attacks.class_gradients` gets every class
gradient of a whole random pool from one backward pass); the reverse-Weibull
maximum-likelihood fit runs on the host with scipy, as in the reference.
"""
from __future__ import annotations

import numpy as np
import torch
from scipy.special import gammainc
from scipy.stats import weibull_min

from . import attacks as A


def empirical_robustness(model, x: torch.Tensor, attack: str, params: dict | None = None):
    """Mean relative Lp size of the minimal successful adversarial perturbation.

    Returns ``(score, adv_x)`` (``(0.0, adv_x)`` when no attack succeeds).
    """
    params = dict(params or {})
    norm = params.get("norm", 2)
    fn = A.ATTACKS.get(attack)
    if fn is None:
        raise NotImplementedError(f"{attack} crafting method not supported")
    if attack == "fgsm":
        params.setdefault("minimal", True)
        params.setdefault("eps_step", 0.1)
        params.setdefault("eps_max", 1.0)
    elif attack == "pgd":
        params.setdefault("minimal", True)
    elif attack == "cw":
        params.pop("norm", None)
        params.pop("targeted", None)
    x = x.detach().float()
    y = A.predict(model, x).argmax(-1)
    adv = fn(model, x, y, **params)
    y_adv = A.predict(model, adv).argmax(-1)
    idx = y_adv != y
    if int(idx.sum()) == 0:
        return 0.0, adv
    n = norm if attack != "cw" else 2
    pert = A._flat_norm(adv[idx] - x[idx], n)
    base = A._flat_norm(x[idx], n)
    return float((pert / base.clamp_min(1e-12)).mean()), adv


def loss_sensitivity(model, x: torch.Tensor, y: torch.Tensor) -> float:
    g = A.loss_gradient(model, x, y)
    return float(g.reshape(g.shape[0], -1).norm(dim=1).mean())


def random_sphere(nb_points: int, nb_dims: int, radius: float, norm, rng: np.random.Generator) -> np.ndarray:
    """Uniform samples in the Lp ball (L2: Gaussian direction x radius U^(1/d) law)."""
    if norm == 2:
        a = rng.standard_normal((nb_points, nb_dims))
        s2 = (a ** 2).sum(1)
        base = gammainc(nb_dims / 2.0, s2 / 2.0) ** (1 / nb_dims) * radius / np.sqrt(s2)
        return a * base[:, None]
    if norm in (np.inf, float("inf")):
        return rng.uniform(-radius, radius, (nb_points, nb_dims))
    if norm == 1:
        a = rng.exponential(1.0, (nb_points, nb_dims)) * rng.choice([-1, 1], (nb_points, nb_dims))
        r = rng.uniform(0, 1, (nb_points, 1)) ** (1 / nb_dims)
        return a / np.abs(a).sum(1, keepdims=True) * r * radius
    raise ValueError(f"norm {norm} not supported")


def _weibull_loc(values: np.ndarray, c_init: float) -> float:
    _, loc, _ = weibull_min.fit(-np.asarray(values, dtype=np.float64), c_init, optimizer=_fmin)
    return float(loc)


def _fmin(func, x0, args, disp=False):
    from scipy.optimize import fmin

    return fmin(func, x0, args=args, xtol=1e-6, maxfun=1000, disp=disp)


def clever_scores(model, x: torch.Tensor, nb_batches: int, batch_size: int, radius: float, norm=2,
                  targets=None, c_init: float = 1.0, pool_factor: int = 10, clip=None,
                  rng: np.random.Generator | None = None) -> dict:
    """CLEVER targeted scores of ONE sample ``x`` for every target class (or ``targets``)."""
    rng = rng or np.random.default_rng(0)
    xs = x.detach().float()
    z0 = A.predict(model, xs.unsqueeze(0))[0]
    pred = int(z0.argmax())
    nc = z0.shape[0]
    tgt = [j for j in (range(nc) if targets is None else targets) if j != pred]
    dim = xs.numel()
    n_pool = pool_factor * batch_size
    pool = random_sphere(n_pool, dim, radius, norm, rng).reshape((n_pool,) + tuple(xs.shape))
    pool = torch.as_tensor(pool, dtype=torch.float32, device=xs.device) + xs.unsqueeze(0)
    if clip is not None:
        pool = pool.clamp(*clip)
    grads = A.class_gradients(model, pool)                    # [P, C, ...]
    gp = grads[:, pred]
    q = np.inf if norm == 1 else (1 if norm in (np.inf, float("inf")) else 2)   # dual norm
    out = {}
    for j in tgt:
        diff = (gp - grads[:, j]).reshape(n_pool, -1)
        if q == 2:
            gn = diff.norm(dim=1)
        elif q == 1:
            gn = diff.abs().sum(1)
        else:
            gn = diff.abs().amax(1)
        gn = gn.cpu().numpy()
        maxes = [gn[rng.choice(n_pool, batch_size)].max() for _ in range(nb_batches)]
        loc = _weibull_loc(np.array(maxes), c_init)
        value = float(z0[pred] - z0[j])
        out[j] = min(-value / loc, radius) if loc != 0 else radius
    return out


def clever_t(model, x, target_class, nb_batches, batch_size, radius, norm=2, c_init=1.0, pool_factor=10, **kw):
    return clever_scores(model, x, nb_batches, batch_size, radius, norm, [target_class], c_init, pool_factor, **kw)[
        target_class]


def clever_u(model, x, nb_batches, batch_size, radius, norm=2, c_init=1.0, pool_factor=10, **kw) -> float:
    s = clever_scores(model, x, nb_batches, batch_size, radius, norm, None, c_init, pool_factor, **kw)
    return float(min(s.values())) if s else float(radius)


def clever(model, x, nb_batches, batch_size, radius, norm=2, target=None, c_init=1.0, pool_factor=10, **kw):
    targets = None if target is None else ([target] if isinstance(target, int) else list(target))
    s = clever_scores(model, x, nb_batches, batch_size, radius, norm, targets, c_init, pool_factor, **kw)
    return np.array([s.get(j) for j in sorted(s)])
