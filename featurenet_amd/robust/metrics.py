"""Robustness metrics: empirical robustness, loss sensitivity and CLEVER.

Reference: the vendored ART metrics module ``model/metrics.py:57-324``
(``empirical_robustness``, ``loss_sensitivity``, ``clever``, ``clever_u``,
``clever_t``).  Gradients are computed in batches on the GPU
(CLEVER: every (sample, target) problem draws its own pool and batches from one generator in
the reference's order, and the gradients of many problems' pools come from one backward pass,
each point seeding its own logit difference); the reverse-Weibull maximum-likelihood fits of
every (sample, target) problem run in one batched call of the native runtime (scipy's exact
estimator in C++, ``csrc/runtime/weibull.cpp``).
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


def _pair_gradients(model, pts: torch.Tensor, seeds: torch.Tensor) -> torch.Tensor:
    """d(z . seed)/dx for every row of ``pts`` [B, ...] with its own logit seed [B, nc]: with seed
    = e_pred - e_target this is grad_pred - grad_target of the reference's ``clever_t``
    (``model/metrics.py:305-309``) in ONE backward pass, parameter gradients off."""
    xg = pts.detach().float().clone().requires_grad_(True)
    with A.no_param_grad(model):
        z = A._logits(model, xg)
        (g,) = torch.autograd.grad(z, xg, grad_outputs=seeds.to(z.dtype))
    return g


def clever_batch(model, xs: torch.Tensor, nb_batches: int, batch_size: int, radius: float, norm=2,
                 targets=None, c_init: float = 1.0, pool_factor: int = 10, clip=None, seed: int = 0,
                 rng=None, chunk_points: int | None = None) -> list[dict]:
    """CLEVER targeted scores of EVERY sample of ``xs`` [S, ...] for every target class (or
    ``targets``): one list entry ``{target: score}`` per sample.

    Reference semantics (``model/metrics.py:205-324`` driven by ``tensorflow_generator.py:
    200-201``): for each sample, for each target class j != pred in class order, ``clever_t``
    draws a FRESH pool of ``pool_factor * batch_size`` points in the Lp ball around the sample
    (``random_sphere``), then ``nb_batches`` index batches of ``batch_size`` from that pool, all
    from ONE global generator that runs on across targets and samples; the estimate is the
    reverse-Weibull location of the per-batch maxima of ||grad_pred - grad_j||_q.  Here the
    generator is ``rng`` (default ``np.random.default_rng(seed)``; pass
    ``np.random.RandomState(s)`` for the reference's legacy ``np.random`` stream -- same calls, same
    order, so the same pools and batches) and the draws follow exactly that order, but the
    gradients of many (sample, target) pools run as one batched backward per chunk (each pool
    point seeds its own logit difference e_pred - e_j, so one pass gives grad_pred - grad_j), the
    next chunk's draws are made while the GPU works on the current one, and every (sample,
    target) fit runs in ONE native batched call."""
    xs = xs.detach().float()
    S = xs.shape[0]
    if S == 0:
        return []
    rng = np.random.default_rng(seed) if rng is None else rng
    z0 = A.predict(model, xs)                                   # [S, nc]
    preds = z0.argmax(-1).tolist()
    nc = z0.shape[1]
    dim = xs[0].numel()
    n_pool = pool_factor * batch_size
    probs = [(s_i, j) for s_i in range(S) for j in (range(nc) if targets is None else targets) if j != preds[s_i]]
    Q = len(probs)
    q = _dual(norm)
    # pool points per backward pass: ~64 MB of fp32 inputs (whole pools per chunk)
    cp = chunk_points or max(n_pool, (16 << 20) // max(dim, 1))
    per = max(1, cp // n_pool)
    dev = xs.device
    maxes = np.zeros((Q, nb_batches), dtype=np.float64)

    def draw(lo: int, hi: int):
        pools = np.empty((hi - lo, n_pool, dim), dtype=np.float32)
        picks = np.empty((hi - lo, nb_batches, batch_size), dtype=np.int64)
        for k in range(hi - lo):                  # the reference's order: pool, then the batches
            pools[k] = random_sphere(n_pool, dim, radius, norm, rng)
            for b in range(nb_batches):
                picks[k, b] = rng.choice(n_pool, batch_size)
        return pools, picks

    def launch(lo: int, hi: int, pools: np.ndarray):
        si = torch.as_tensor([probs[k][0] for k in range(lo, hi)], device=dev)
        tj = torch.as_tensor([probs[k][1] for k in range(lo, hi)], device=dev)
        pts = torch.as_tensor(pools, device=dev).reshape((hi - lo, n_pool) + tuple(xs.shape[1:]))
        pts = (pts + xs[si].unsqueeze(1)).reshape(((hi - lo) * n_pool,) + tuple(xs.shape[1:]))
        if clip is not None:
            pts = pts.clamp(*clip)
        sd = torch.zeros(hi - lo, nc, device=dev)
        r = torch.arange(hi - lo, device=dev)
        sd[r, torch.as_tensor(preds, device=dev)[si]] = 1.0
        sd[r, tj] -= 1.0
        g = _pair_gradients(model, pts, sd.repeat_interleave(n_pool, 0)).reshape(hi - lo, n_pool, -1)
        if q == 2:
            return g.norm(dim=-1)
        return g.abs().sum(-1) if q == 1 else g.abs().amax(-1)

    pending = None
    lo = 0
    nxt = draw(0, min(per, Q)) if Q else None
    while lo < Q:
        hi = min(lo + per, Q)
        pools, picks = nxt
        gn = launch(lo, hi, pools)                # (asynchronous on the GPU)
        if hi < Q:
            nxt = draw(hi, min(hi + per, Q))      # the next chunk's draws overlap this chunk's pass
        if pending is not None:
            plo, phi, pg, pp = pending
            maxes[plo:phi] = np.take_along_axis(pg.double().cpu().numpy()[:, None, :],
                                                pp.reshape(phi - plo, 1, -1), 2).reshape(
                phi - plo, nb_batches, batch_size).max(-1)
        pending = (lo, hi, gn, picks)
        lo = hi
    if pending is not None:
        plo, phi, pg, pp = pending
        maxes[plo:phi] = np.take_along_axis(pg.double().cpu().numpy()[:, None, :], pp.reshape(phi - plo, 1, -1),
                                            2).reshape(phi - plo, nb_batches, batch_size).max(-1)
    locs = weibull_locs(maxes, c_init) if Q else np.zeros(0)
    z0c = z0.double().cpu().numpy()
    out: list[dict] = [dict() for _ in range(S)]
    for (s_i, j), loc in zip(probs, locs):
        value = float(z0c[s_i, preds[s_i]] - z0c[s_i, j])
        out[s_i][j] = min(-value / loc, radius) if loc != 0 else radius
    return out


def clever_scores(model, x: torch.Tensor, nb_batches: int, batch_size: int, radius: float, norm=2,
                  targets=None, c_init: float = 1.0, pool_factor: int = 10, clip=None, rng=None) -> dict:
    """CLEVER targeted scores of ONE sample ``x`` for every target class (or ``targets``); ``rng``
    (optional) is the generator the draws continue from (the reference's global stream)."""
    return clever_batch(model, x.unsqueeze(0), nb_batches, batch_size, radius, norm, targets, c_init, pool_factor,
                        clip, rng=rng)[0]


def clever_t_literal(model, x: torch.Tensor, target: int, nb_batches: int, batch_size: int, radius: float, norm,
                     c_init: float, pool_factor: int, clip, rng) -> float:
    """The reference's ``clever_t`` line by line (``model/metrics.py:242-324``): pool, batches,
    class gradients of each batch, per-batch max norm, reverse-Weibull fit -- one target of one
    sample, unbatched.  The test oracle of :func:`clever_batch`."""
    xs = x.detach().float()
    z0 = A.predict(model, xs.unsqueeze(0))[0].double()
    pred = int(z0.argmax())
    if target == pred:
        raise ValueError("The targeted class is the predicted class.")
    dim = xs.numel()
    n_pool = pool_factor * batch_size
    pool = random_sphere(n_pool, dim, radius, norm, rng).astype(np.float32).reshape((n_pool,) + tuple(xs.shape))
    pool = torch.as_tensor(pool, device=xs.device) + xs.unsqueeze(0)
    if clip is not None:
        pool = pool.clamp(*clip)
    q = _dual(norm)
    gmax = []
    for _ in range(nb_batches):
        pick = torch.as_tensor(rng.choice(n_pool, batch_size), device=xs.device)
        grads = A.class_gradients(model, pool[pick])              # [bs, C, ...]
        d = (grads[:, pred] - grads[:, target]).reshape(batch_size, -1)
        gn = d.norm(dim=1) if q == 2 else (d.abs().sum(1) if q == 1 else d.abs().amax(1))
        gmax.append(float(gn.max()))
    loc = _weibull_loc(np.asarray(gmax), c_init)
    value = float(z0[pred] - z0[target])
    return min(-value / loc, radius) if loc != 0 else radius


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
