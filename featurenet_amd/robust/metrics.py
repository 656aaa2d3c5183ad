"""Robustness metrics: empirical robustness, loss sensitivity and CLEVER.

Reference: the vendored ART metrics module ``model/metrics.py:57-324``
(``empirical_robustness``, ``loss_sensitivity``, ``clever``, ``clever_u``,
``clever_t``).  Gradients are computed in batches on the GPU
(:func:`featurenet_amd.robust.attacks.class_gradients` gets every class
gradient of a whole random pool from one backward pass); the reverse-Weibull
maximum-likelihood fits of every (sample, target) problem run in one batched call of the
native runtime (scipy's exact estimator in C++, ``csrc/runtime/weibull.cpp``).
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
    return float(weibull_locs(np.asarray(values, dtype=np.float64)[None, :], c_init)[0])


def _fmin(func, x0, args, disp=False):
    from scipy.optimize import fmin

    return fmin(func, x0, args=args, xtol=1e-6, maxfun=1000, disp=disp)


def weibull_locs(maxes: np.ndarray, c_init: float = 1.0) -> np.ndarray:
    """Location of the reverse-Weibull MLE fit of every row of ``maxes`` [Q, nb_batches]
    (reference: ``weibull_min.fit(-maxes, c_init, optimizer=fmin)``, ``model/metrics.py``
    ``clever_t``).  The native runtime runs scipy's exact estimator (same start point,
    likelihood and Nelder-Mead steps; ``csrc/runtime/weibull.cpp``) for all rows on a thread
    pool -- ~0.3 ms per fit instead of ~35 ms of Python-level scipy; scipy is the fallback."""
    from .. import _native
    from scipy.stats import weibull_min

    data = -np.ascontiguousarray(maxes, dtype=np.float64)
    if data.ndim != 2:
        raise ValueError("maxes must be [problems, values]")
    if _native.runtime_available():
        fit = _native.runtime().weibull_min_fit_batch(data, float(c_init), 1e-6, 1e-4, 1000, 0)
        if not (np.all(fit[:, 0] > 0) and np.all(fit[:, 2] > 0)):   # scipy raises FitError there
            raise RuntimeError("reverse-Weibull fit converged outside the distribution's parameter range")
        return fit[:, 1].copy()
    return np.array([weibull_min.fit(row, c_init, optimizer=_fmin)[1] for row in data], dtype=np.float64)


def _dual(norm):
    return np.inf if norm == 1 else (1 if norm in (np.inf, float("inf")) else 2)


def clever_batch(model, xs: torch.Tensor, nb_batches: int, batch_size: int, radius: float, norm=2,
                 targets=None, c_init: float = 1.0, pool_factor: int = 10, clip=None, seed: int = 0,
                 chunk_samples: int | None = None) -> list[dict]:
    """CLEVER targeted scores of EVERY sample of ``xs`` [S, ...] for every target class (or
    ``targets``): one list entry ``{target: score}`` per sample.

    The reference loops over samples (``tensorflow_generator.py:182-203``), each with a fresh
    generator seeded 0 (one random pool of ``pool_factor * batch_size`` points in the Lp ball
    and ``nb_batches`` random batches per target), a class-gradient pass of its pool and one
    reverse-Weibull fit per target.  Here the same draws (every sample's generator starts at
    seed 0, so the pool directions and batch indices are shared) feed batched gradient passes
    over many samples' pools at once (:func:`~featurenet_amd.robust.attacks.class_gradients`,
    parameter gradients off) and ONE batched fit of every (sample, target) problem."""
    xs = xs.detach().float()
    S = xs.shape[0]
    if S == 0:
        return []
    z0 = A.predict(model, xs)                                   # [S, nc]
    preds = z0.argmax(-1).tolist()
    nc = z0.shape[1]
    dim = xs[0].numel()
    n_pool = pool_factor * batch_size
    rng = np.random.default_rng(seed)
    sphere = random_sphere(n_pool, dim, radius, norm, rng).reshape((n_pool,) + tuple(xs.shape[1:]))
    sphere = torch.as_tensor(sphere, dtype=torch.float32, device=xs.device)
    tgts = [[j for j in (range(nc) if targets is None else targets) if j != p] for p in preds]
    ntg = max((len(t) for t in tgts), default=0)
    # the batches each target position draws from a seed-0 generator after the pool
    choice = np.stack([np.stack([rng.choice(n_pool, batch_size) for _ in range(nb_batches)]) for _ in range(ntg)]) \
        if ntg else np.zeros((0, nb_batches, batch_size), dtype=np.int64)
    q = _dual(norm)
    step = chunk_samples or max(1, 16384 // max(n_pool * nc, 1))
    norms = np.zeros((S, nc, n_pool), dtype=np.float64)          # ||grad_pred - grad_j|| over the pool
    for i in range(0, S, step):
        xb = xs[i:i + step]
        b = xb.shape[0]
        pool = (sphere.unsqueeze(0) + xb.unsqueeze(1)).reshape((b * n_pool,) + tuple(xs.shape[1:]))
        if clip is not None:
            pool = pool.clamp(*clip)
        g = A.class_gradients(model, pool).reshape(b, n_pool, nc, -1)   # [b, P, C, dim]
        pr = torch.as_tensor(preds[i:i + b], device=xs.device)
        gp = g[torch.arange(b, device=xs.device), :, pr]            # [b, P, dim]
        diff = gp.unsqueeze(2) - g                                  # [b, P, C, dim]
        if q == 2:
            gn = diff.norm(dim=-1)
        elif q == 1:
            gn = diff.abs().sum(-1)
        else:
            gn = diff.abs().amax(-1)
        norms[i:i + b] = gn.permute(0, 2, 1).double().cpu().numpy()
    rows, keys = [], []
    for s_i in range(S):
        for t, j in enumerate(tgts[s_i]):
            gn = norms[s_i, j]
            rows.append([gn[choice[t, k]].max() for k in range(nb_batches)])
            keys.append((s_i, j))
    locs = weibull_locs(np.asarray(rows, dtype=np.float64), c_init) if rows else np.zeros(0)
    z0c = z0.double().cpu().numpy()
    out: list[dict] = [dict() for _ in range(S)]
    for (s_i, j), loc in zip(keys, locs):
        value = float(z0c[s_i, preds[s_i]] - z0c[s_i, j])
        out[s_i][j] = min(-value / loc, radius) if loc != 0 else radius
    return out


def clever_scores(model, x: torch.Tensor, nb_batches: int, batch_size: int, radius: float, norm=2,
                  targets=None, c_init: float = 1.0, pool_factor: int = 10, clip=None,
                  rng: np.random.Generator | None = None) -> dict:
    """CLEVER targeted scores of ONE sample ``x`` for every target class (or ``targets``)."""
    if rng is not None:
        return _clever_scores_rng(model, x, nb_batches, batch_size, radius, norm, targets, c_init, pool_factor, clip,
                                  rng)
    return clever_batch(model, x.unsqueeze(0), nb_batches, batch_size, radius, norm, targets, c_init, pool_factor,
                        clip)[0]


def _clever_scores_rng(model, x, nb_batches, batch_size, radius, norm, targets, c_init, pool_factor, clip, rng):
    """One sample with a caller-supplied generator (its draws continue across calls)."""
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
    q = _dual(norm)
    rows = []
    for j in tgt:
        diff = (gp - grads[:, j]).reshape(n_pool, -1)
        gn = (diff.norm(dim=1) if q == 2 else diff.abs().sum(1) if q == 1 else diff.abs().amax(1)).cpu().numpy()
        rows.append([gn[rng.choice(n_pool, batch_size)].max() for _ in range(nb_batches)])
    locs = weibull_locs(np.asarray(rows, dtype=np.float64), c_init) if rows else []
    out = {}
    for j, loc in zip(tgt, locs):
        value = float(z0[pred] - z0[j])
        out[j] = min(-value / loc, radius) if loc != 0 else radius
    return out


def clever_t(model, x, target_class, nb_batches, batch_size, radius, norm=2, c_init=1.0, pool_factor=10, **kw):
    return clever_scores(model, x, nb_batches, batch_size, radius, norm, [target_class], c_init, pool_factor, **kw)[
        target_class]


def clever_u(model, x, nb_batches, batch_size, radius, norm=2, c_init=1.0, pool_factor=10, **kw) -> float:
    s = clever_scores(model, x, nb_batches, batch_size, radius, norm, None, c_init, pool_factor, **kw)
    return float(min(s.values())) if s else float(radius)


def clever_u_batch(model, xs, nb_batches, batch_size, radius, norm=2, c_init=1.0, pool_factor=10, clip=None,
                   **kw) -> np.ndarray:
    """Untargeted CLEVER of every sample of ``xs`` (= :func:`clever_u` per sample, batched)."""
    res = clever_batch(model, xs, nb_batches, batch_size, radius, norm, None, c_init, pool_factor, clip, **kw)
    return np.array([min(s.values()) if s else float(radius) for s in res], dtype=np.float64)


def clever(model, x, nb_batches, batch_size, radius, norm=2, target=None, c_init=1.0, pool_factor=10, **kw):
    targets = None if target is None else ([target] if isinstance(target, int) else list(target))
    s = clever_scores(model, x, nb_batches, batch_size, radius, norm, targets, c_init, pool_factor, **kw)
    return np.array([s.get(j) for j in sorted(s)])
