"""Adversarial attacks, batched on the GPU through the native kernels' autograd.

Reference: the ART 0.9 attacks the reference wires in ``model/metrics.py:38-43``
(FastGradientMethod, ProjectedGradientDescent, CarliniL2Method) with the
parameters of ``tensorflow_generator.py:151-173`` (norm 2; PGD eps 1, step
0.1; CW untargeted; "minimal" perturbation search for empirical robustness).
Input gradients flow through the same HIP kernels as training (the conv
dgrad kernel computes d(loss)/d(input)); every attack runs on whole batches,
not per-sample Python loops.

Attacks need d(loss)/d(input) only: every gradient here is taken under
:func:`no_param_grad`, so the conv / dense backward never launches a weight-gradient kernel
(``needs_input_grad`` of the weights is False) and nothing is written into the training
gradient buffer (``FlatParams`` slots) -- about a third of each PGD / CW / CLEVER iteration's
kernels in round 3.
"""
from __future__ import annotations

import contextlib
import math

import torch
import torch.nn.functional as F


def _logits(model, x: torch.Tensor) -> torch.Tensor:
    return model(x).float()


@contextlib.contextmanager
def no_param_grad(model):
    """Input-gradient-only autograd through ``model``: parameters stop requiring grad for the
    duration (restored on exit, also after an exception)."""
    ps = [p for p in model.parameters() if p.requires_grad]
    for p in ps:
        p.requires_grad_(False)
    try:
        yield
    finally:
        for p in ps:
            p.requires_grad_(True)


def predict(model, x: torch.Tensor, batch_size: int = 256) -> torch.Tensor:
    outs = []
    with torch.no_grad():
        for i in range(0, len(x), batch_size):
            outs.append(_logits(model, x[i:i + batch_size]))
    return torch.cat(outs)


def _flat_norm(t: torch.Tensor, norm) -> torch.Tensor:
    f = t.reshape(t.shape[0], -1)
    if norm == 2:
        return f.norm(dim=1)
    if norm == 1:
        return f.abs().sum(1)
    return f.abs().amax(1)


def _direction(g: torch.Tensor, norm) -> torch.Tensor:
    """Steepest-ascent unit step for the given norm (FGM)."""
    if norm in (float("inf"), "inf", math.inf):
        return g.sign()
    shape = (-1,) + (1,) * (g.dim() - 1)
    if norm == 1:
        return g / (g.reshape(g.shape[0], -1).abs().sum(1).reshape(shape) + 1e-12)
    return g / (g.reshape(g.shape[0], -1).norm(dim=1).reshape(shape) + 1e-12)


def loss_gradient(model, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    xg = x.detach().float().clone().requires_grad_(True)
    with no_param_grad(model):
        loss = F.cross_entropy(_logits(model, xg), y, reduction="sum")
        (g,) = torch.autograd.grad(loss, xg)
    return g


def class_gradients(model, x: torch.Tensor, classes: torch.Tensor | None = None,
                    max_rows: int = 16384) -> torch.Tensor:
    """d logit_c / d x for every class c (or the listed ones): [B, C, *x.shape[1:]].

    All classes are obtained from ONE backward pass per chunk: the batch is replicated per
    class and each replica back-propagates its own one-hot seed; chunks of at most
    ``max_rows`` replicated rows bound the activation memory of large pools (CLEVER over a
    whole robustness set)."""
    B = x.shape[0]
    with torch.no_grad():
        nc = _logits(model, x[:1]).shape[-1]
    cls = torch.arange(nc, device=x.device) if classes is None else classes.to(x.device)
    C = len(cls)
    step = max(1, max_rows // max(C, 1))
    out = []
    with no_param_grad(model):
        for i in range(0, B, step):
            xb = x[i:i + step].detach().float()
            b = xb.shape[0]
            xr = xb.unsqueeze(1).expand(b, C, *x.shape[1:]).reshape(b * C, *x.shape[1:]).clone()
            xr.requires_grad_(True)
            z = _logits(model, xr)
            seed = torch.zeros_like(z)
            seed[torch.arange(b * C, device=x.device), cls.repeat(b)] = 1.0
            (g,) = torch.autograd.grad(z, xr, grad_outputs=seed)
            out.append(g.reshape(b, C, *x.shape[1:]))
    return out[0] if len(out) == 1 else torch.cat(out)


def fgsm(model, x: torch.Tensor, y: torch.Tensor | None = None, eps: float = 0.3, norm=float("inf"),
         clip=(0.0, 1.0), minimal: bool = False, eps_step: float = 0.1, eps_max: float = 1.0) -> torch.Tensor:
    """Fast gradient method.  ``minimal`` grows eps by ``eps_step`` up to
    ``eps_max`` per sample until it is misclassified (ART semantics)."""
    x = x.detach().float()
    if y is None:
        y = predict(model, x).argmax(-1)
    d = _direction(loss_gradient(model, x, y), norm)
    if not minimal:
        return (x + eps * d).clamp(*clip) if clip else x + eps * d
    adv = x.clone()
    done = torch.zeros(len(x), dtype=torch.bool, device=x.device)
    e = eps_step
    while e <= eps_max + 1e-9 and not bool(done.all()):
        cand = x + e * d
        if clip:
            cand = cand.clamp(*clip)
        pred = predict(model, cand).argmax(-1)
        newly = (~done) & (pred != y)
        shape = (-1,) + (1,) * (x.dim() - 1)
        adv = torch.where(newly.reshape(shape), cand, adv)
        done |= newly
        e += eps_step
    return adv


def _project(delta: torch.Tensor, eps: float, norm) -> torch.Tensor:
    if norm in (float("inf"), "inf", math.inf):
        return delta.clamp(-eps, eps)
    n = _flat_norm(delta, norm).reshape((-1,) + (1,) * (delta.dim() - 1))
    return delta * torch.clamp(eps / (n + 1e-12), max=1.0)


def pgd(model, x: torch.Tensor, y: torch.Tensor | None = None, eps: float = 1.0, eps_step: float = 0.1,
        max_iter: int = 100, norm=2, clip=(0.0, 1.0), random_init: bool = False, minimal: bool = True) -> torch.Tensor:
    """Projected gradient descent (untargeted).  ``minimal`` keeps, per sample,
    the first iterate that flips the prediction (smallest perturbation found)."""
    x = x.detach().float()
    if y is None:
        y = predict(model, x).argmax(-1)
    delta = torch.zeros_like(x)
    if random_init:
        delta = _project(torch.empty_like(x).uniform_(-eps, eps), eps, norm)
    best = x.clone()
    done = torch.zeros(len(x), dtype=torch.bool, device=x.device)
    shape = (-1,) + (1,) * (x.dim() - 1)
    for _ in range(max_iter):
        xa = x + delta
        if clip:
            xa = xa.clamp(*clip)
        g = loss_gradient(model, xa, y)
        delta = _project(delta + eps_step * _direction(g, norm), eps, norm)
        xa = (x + delta).clamp(*clip) if clip else x + delta
        pred = predict(model, xa).argmax(-1)
        if minimal:
            newly = (~done) & (pred != y)
            best = torch.where(newly.reshape(shape), xa, best)
            done |= newly
            if bool(done.all()):
                break
        else:
            best = xa
    if minimal:
        best = torch.where(done.reshape(shape), best, (x + delta).clamp(*clip) if clip else x + delta)
    return best


def carlini_l2(model, x: torch.Tensor, y: torch.Tensor | None = None, confidence: float = 0.0,
               learning_rate: float = 0.01, binary_search_steps: int = 10, max_iter: int = 10,
               initial_const: float = 0.01, clip=(0.0, 1.0)) -> torch.Tensor:
    """Carlini & Wagner L2 (untargeted), tanh change of variables + Adam, binary
    search on the trade-off constant (ART 0.9 defaults)."""
    x = x.detach().float()
    if y is None:
        y = predict(model, x).argmax(-1)
    lo, hi = clip if clip else (float(x.min()), float(x.max()))
    span = max(hi - lo, 1e-6)
    B = len(x)
    shape = (-1,) + (1,) * (x.dim() - 1)
    x01 = ((x - lo) / span).clamp(1e-6, 1 - 1e-6)
    w0 = torch.atanh(2 * x01 - 1)
    c = torch.full((B,), initial_const, device=x.device)
    c_lo = torch.zeros(B, device=x.device)
    c_hi = torch.full((B,), 1e10, device=x.device)
    best_l2 = torch.full((B,), float("inf"), device=x.device)
    best_adv = x.clone()
    nc = predict(model, x[:1]).shape[-1]
    onehot = F.one_hot(y, nc).float()
    with no_param_grad(model):
        return _cw_search(model, x, y, confidence, learning_rate, binary_search_steps, max_iter, lo, span, B, shape,
                          w0, c, c_lo, c_hi, best_l2, best_adv, onehot)


def _cw_search(model, x, y, confidence, learning_rate, binary_search_steps, max_iter, lo, span, B, shape, w0, c,
               c_lo, c_hi, best_l2, best_adv, onehot):
    for _ in range(binary_search_steps):
        w = w0.clone().requires_grad_(True)
        opt = torch.optim.Adam([w], lr=learning_rate)
        succeeded = torch.zeros(B, dtype=torch.bool, device=x.device)
        for _ in range(max_iter):
            adv = lo + span * (torch.tanh(w) + 1) / 2
            z = _logits(model, adv)
            real = (z * onehot).sum(1)
            other = (z - 1e9 * onehot).amax(1)
            f = torch.clamp(real - other + confidence, min=0.0)
            l2 = ((adv - x) ** 2).reshape(B, -1).sum(1)
            loss = (l2 + c * f).sum()
            # gradient w.r.t. the attack variable only (and no parameter requires grad: no
            # weight-gradient kernels, no writes into the training gradient buffer, no DP hooks)
            (w.grad,) = torch.autograd.grad(loss, [w])
            opt.step()
            with torch.no_grad():
                ok = (z.argmax(1) != y) & (f <= 0)
                better = ok & (l2 < best_l2)
                best_l2 = torch.where(better, l2.detach(), best_l2)
                best_adv = torch.where(better.reshape(shape), adv.detach(), best_adv)
                succeeded |= ok
        with torch.no_grad():
            c_hi = torch.where(succeeded, torch.minimum(c_hi, c), c_hi)
            c_lo = torch.where(~succeeded, torch.maximum(c_lo, c), c_lo)
            c = torch.where(c_hi < 1e9, (c_lo + c_hi) / 2, c * 10)
    return best_adv


ATTACKS = {"fgsm": fgsm, "pgd": pgd, "cw": carlini_l2}
