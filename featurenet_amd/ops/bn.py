"""BatchNorm(+activation) and BN+act+pool ops.

Reference parity: Keras ``BatchNormalization`` (``model/operation.py:139-150``,
axis forced to 1 there -- see :mod:`featurenet_amd.ir.compile` for the compat
flag) and the north-star BatchNorm3d+ReLU(+MaxPool3d) block of FeatureNet-3D.

GPU path: statistics come either from the producing conv's epilogue slab
(no extra pass over ``y``) or from ``colstats``; ``bn_finalize`` reduces the
slab in fp64; ``bn_apply`` (or ``pool_fwd`` with the BN prologue) writes the
normalised activation.  Backward is two passes over ``y``: ``colstats``
(mode 1) for (sum g, sum g*xhat) and ``bn_bwd_apply``.
"""
from __future__ import annotations

import torch

from .. import _native
from ..training.flat import grad_target
from . import bnfuse
from . import reference as ref
from .spec import PoolSpec, act_code


def _stats_slab(y2: torch.Tensor) -> torch.Tensor:
    M, C = y2.shape
    nb = _native.kernels().colstats_blocks(M, C, 0, 0)
    part = torch.empty(nb, 2, C, dtype=torch.float32, device=y2.device)
    _native.kernels().colstats(y2.data_ptr(), 0, 0, 0, 0, 0, part.data_ptr(), M, C, 0, 0, nb, _native.stream(y2))
    return part


def _finalize_fwd(slab, count, gamma, beta, rmean, rvar, momentum, eps, update_running=True):
    C = slab.shape[-1]
    out = torch.empty(4, C, dtype=torch.float32, device=slab.device)
    _native.kernels().bn_finalize(
        slab.data_ptr(), slab.shape[0], C, float(count), _native.ptr(gamma), _native.ptr(beta),
        _native.ptr(rmean) if update_running else 0, _native.ptr(rvar) if update_running else 0,
        float(momentum), float(eps), out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), out[3].data_ptr(), 0,
        _native.stream(slab))
    return out  # mean, invstd, scale, shift


def _eval_params(gamma, beta, rmean, rvar, eps, C, device):
    g = gamma.detach().float() if gamma is not None else torch.ones(C, device=device)
    b = beta.detach().float() if beta is not None else torch.zeros(C, device=device)
    invstd = torch.rsqrt(rvar.float() + eps)
    scale = g * invstd
    shift = b - rmean.float() * scale
    return torch.stack([rmean.float(), invstd, scale, shift])


def _bwd_param_grads(dz2, y2, prm, act, beta=None, gamma=None, part=None):
    """(dbeta, dgamma) = (sum g, sum g*xhat), written straight into the parameters' flat
    gradients when :func:`grad_target` offers them.  ``part``: per-block partial sums
    [nb, 2, C] of the raw backward moments (sum g, sum g*y) already produced by the pass that
    wrote dz (the max-pool backward, the pointwise head's dgrad); otherwise ``colstats``
    computes them."""
    M, C = y2.shape
    K = _native.kernels()
    st = _native.stream(y2)
    mode = 2                                     # raw moments (sum g, sum g*y)
    if part is None:
        mode = 1                                 # colstats: (sum g, sum g*xhat)
        nb = K.colstats_blocks(M, C, 1, act)
        part = torch.empty(nb, 2, C, dtype=torch.float32, device=y2.device)
        K.colstats(y2.data_ptr(), dz2.data_ptr(), prm[2].data_ptr(), prm[3].data_ptr(), prm[0].data_ptr(),
                   prm[1].data_ptr(), part.data_ptr(), M, C, act, 1, nb, st)
    nb = part.shape[0]
    db, dg = grad_target(beta), grad_target(gamma)
    if db is None or dg is None or db.numel() != C or dg.numel() != C:
        out = torch.empty(2, C, dtype=torch.float32, device=y2.device)
        db, dg = out[0], out[1]
    K.bn_finalize(part.data_ptr(), nb, C, float(M), 0, 0, prm[0].data_ptr() if mode == 2 else 0,
                  prm[1].data_ptr() if mode == 2 else 0, 0.0, 0.0, db.data_ptr(), dg.data_ptr(), 0, 0, mode, st)
    return db, dg


def _bwd_identity(g2, y2, prm, beta, gamma, gslab, wpart):
    """BN(+relu) backward from the statistics identity (``bn_pool.hip`` bn_bwd_prep_kernel):
    ``g2`` = dz [M, C] from the consuming conv's dgrad, ``gslab`` the column sums of
    g = dz * relu'(z) its epilogue made
    [nbg, 2, C] (row 0), ``wpart`` the partials of S = sum W . dW [nbw, C].  Returns
    (dy, dbeta, dgamma); dbeta / dgamma go straight into the flat gradients when offered."""
    M, C = y2.shape
    K = _native.kernels()
    st = _native.stream(y2)
    db, dg = grad_target(beta), grad_target(gamma)
    tmp = torch.empty(3, C, dtype=torch.float32, device=y2.device)
    if db is None or db.numel() != C:
        db = tmp[0]
    if dg is None or dg.numel() != C:
        dg = tmp[1]
    kc = torch.empty(3, C, dtype=torch.float32, device=y2.device)
    K.bn_bwd_prep(gslab.data_ptr(), gslab.shape[0], wpart.data_ptr(), wpart.shape[0], C, float(M),
                  _native.ptr(gamma), _native.ptr(beta), prm[0].data_ptr(), prm[1].data_ptr(), prm[2].data_ptr(),
                  prm[3].data_ptr(), db.data_ptr(), kc.data_ptr(), g2.data_ptr(), y2.data_ptr(), M, st,
                  [gslab.numel(), wpart.numel(), kc.numel(), g2.numel(), y2.numel()])
    dy = torch.empty_like(y2)
    nb = K.bn_bwd_apply_k_blocks(M, C)
    part = torch.empty(nb, 2, C, dtype=torch.float32, device=y2.device)
    K.bn_bwd_apply_k(g2.data_ptr(), y2.data_ptr(), kc.data_ptr(), prm[0].data_ptr(), prm[1].data_ptr(),
                     prm[3].data_ptr(), dy.data_ptr(), M, C, part.data_ptr(), nb, st,
                     [g2.numel(), y2.numel(), dy.numel(), part.numel()])
    # dgamma = sum g * xhat, summed exactly from (g, y) by the apply pass (row 1 of its slab)
    K.bn_finalize(part.data_ptr(), nb, C, float(M), 0, 0, 0, 0, 0.0, 0.0, tmp[2].data_ptr(), dg.data_ptr(), 0, 0, 1,
                  st)
    return dy, db, dg


def _bwd_input(dz2, y2, prm, dbeta, dgamma, act, training):
    M, C = y2.shape
    dy = torch.empty_like(y2)
    if training:
        db, dg, inv = dbeta, dgamma, 1.0 / M
    else:                                        # eval: the statistics are constants
        db = dg = torch.zeros(C, dtype=torch.float32, device=y2.device)
        inv = 0.0
    _native.kernels().bn_bwd_apply(dz2.data_ptr(), y2.data_ptr(), prm[2].data_ptr(), prm[3].data_ptr(),
                                   prm[0].data_ptr(), prm[1].data_ptr(), db.data_ptr(), dg.data_ptr(), dy.data_ptr(),
                                   y2.numel(), C, inv, act, _native.stream(y2))
    return dy


class BatchNormActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, gamma, beta, slab, rmean, rvar, training, momentum, eps, act, tag=False, lazy=False):
        C = y.shape[-1]
        y2 = y.reshape(-1, C)
        if training:
            if slab is None:
                slab = _stats_slab(y2)
            prm = _finalize_fwd(slab, y2.shape[0], gamma, beta, rmean, rvar, momentum, eps)
        else:
            prm = _eval_params(gamma, beta, rmean, rvar, eps, C, y.device)
        z = torch.empty_like(y)
        # the relu-mask bytes of the statistics identity (ops/bnfuse.py): the consuming conv's
        # dgrad applies them, so the backward needs no colstats pass
        mask = (torch.empty(y2.numel() // 8, dtype=torch.uint8, device=y.device)
                if tag and bnfuse.identity_ok(C, act) else None)

        def fill():
            _native.kernels().bn_apply(y2.data_ptr(), prm[2].data_ptr(), prm[3].data_ptr(), z.data_ptr(), y2.numel(),
                                       C, act, _native.stream(y), _native.ptr(mask), 0 if mask is None else mask.numel())

        if lazy and act == 1 and C % 8 == 0 and bnfuse.prologue_enabled():
            # the caller's next op is a conv: its conv_tile loader applies BN + act to y's halo and
            # writes z and the mask (ops/bnfuse.py defer / settle), else ``fill`` runs there
            bnfuse.defer(z, y, prm, act, mask, fill)
        else:
            fill()
        if tag and act in (0, 1):                # none / relu: the dgrad epilogue's forms
            bnfuse.tag_output(z, y, prm, act, mask)
        ctx.mask = mask                          # (alive until the backward: the conv's dgrad reads it)
        ctx.save_for_backward(y, prm)
        ctx.act, ctx.training = act, training
        ctx.has_gamma, ctx.has_beta = gamma is not None, beta is not None
        ctx.params = (beta, gamma)                   # leaves: for their direct flat gradients
        return z

    @staticmethod
    def backward(ctx, dz):
        y, prm = ctx.saved_tensors
        C = y.shape[-1]
        y2 = y.reshape(-1, C)
        dz2 = dz.contiguous().to(torch.bfloat16).reshape(-1, C)
        part = bnfuse.take(dz2, y) if ctx.training else None
        ctx.mask = None
        if isinstance(part, tuple) and ctx.needs_input_grad[0]:
            dy, dbeta, dgamma = _bwd_identity(dz2, y2, prm, *ctx.params, gslab=part[1], wpart=part[2])
            return (dy.reshape(y.shape), dgamma if ctx.has_gamma else None, dbeta if ctx.has_beta else None,
                    None, None, None, None, None, None, None, None, None)
        dbeta = dgamma = None
        if ctx.training or ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            # (no identity slab, or no input gradient wanted: the colstats pass.  Eval mode with
            # frozen parameters -- input gradients of robustness attacks -- needs neither)
            dbeta, dgamma = _bwd_param_grads(dz2, y2, prm, ctx.act, *ctx.params)
        dy = _bwd_input(dz2, y2, prm, dbeta, dgamma, ctx.act, ctx.training) if ctx.needs_input_grad[0] else None
        return (None if dy is None else dy.reshape(y.shape), dgamma if ctx.has_gamma else None,
                dbeta if ctx.has_beta else None, None, None, None, None, None, None, None, None, None)


class BatchNormActPoolFn(torch.autograd.Function):
    """p = pool(act(bn(y))) without materialising act(bn(y))."""

    @staticmethod
    def forward(ctx, y, gamma, beta, slab, rmean, rvar, training, momentum, eps, act, pspec, is_max, count_pad):
        C = y.shape[-1]
        y2 = y.reshape(-1, C)
        if training:
            if slab is None:
                slab = _stats_slab(y2)
            prm = _finalize_fwd(slab, y2.shape[0], gamma, beta, rmean, rvar, momentum, eps)
        else:
            prm = _eval_params(gamma, beta, rmean, rvar, eps, C, y.device)
        p = torch.empty(pspec.out_shape5, dtype=torch.bfloat16, device=y.device)
        _native.kernels().pool_fwd(y.data_ptr(), p.data_ptr(), prm[2].data_ptr(), prm[3].data_ptr(), pspec.geom17(),
                                   int(is_max), int(count_pad), act, _native.stream(y), [y.numel(), p.numel()])
        ctx.save_for_backward(y, prm)
        ctx.act, ctx.training, ctx.pspec, ctx.is_max, ctx.count_pad = act, training, pspec, is_max, count_pad
        ctx.has_gamma, ctx.has_beta = gamma is not None, beta is not None
        ctx.params = (beta, gamma)
        return p

    @staticmethod
    def backward(ctx, dp):
        y, prm = ctx.saved_tensors
        C = y.shape[-1]
        dp = dp.contiguous().to(torch.bfloat16)
        K = _native.kernels()
        geom = ctx.pspec.geom17()
        nb = K.pool_bwd_stats_blocks(geom) if (ctx.is_max and ctx.training and bnfuse.pool_stats_enabled()) else 0
        part = None
        ps = ctx.pspec
        if nb > 0 and bnfuse.pool_apply_enabled() and ps.KD * ps.KH * ps.KW <= 8 and C % 8 == 0:
            # the moments without writing dz, then dy straight from (dp, y): no sparse dz pass
            part = torch.empty(nb, 2, C, dtype=torch.float32, device=y.device)
            K.pool_bwd_stats(dp.data_ptr(), y.data_ptr(), 0, prm[2].data_ptr(), prm[3].data_ptr(), geom, ctx.act,
                             part.data_ptr(), _native.stream(y), [y.numel(), dp.numel(), part.numel()])
            y2 = y.reshape(-1, C)
            dbeta, dgamma = _bwd_param_grads(None, y2, prm, ctx.act, *ctx.params, part=part)
            dy = None
            if ctx.needs_input_grad[0]:
                dy = torch.empty_like(y)
                K.pool_bn_bwd_apply(dp.data_ptr(), y.data_ptr(), prm[2].data_ptr(), prm[3].data_ptr(),
                                    prm[0].data_ptr(), prm[1].data_ptr(), dbeta.data_ptr(), dgamma.data_ptr(),
                                    dy.data_ptr(), geom, ctx.act, 1.0 / y2.shape[0], _native.stream(y),
                                    [y.numel(), dp.numel()])
            return (dy, dgamma if ctx.has_gamma else None, dbeta if ctx.has_beta else None) + (None,) * 10
        dz = torch.empty_like(y)
        if nb > 0:
            # max-pool backward + this BN's raw backward moments in one pass (no colstats)
            part = torch.empty(nb, 2, C, dtype=torch.float32, device=y.device)
            K.pool_bwd_stats(dp.data_ptr(), y.data_ptr(), dz.data_ptr(), prm[2].data_ptr(), prm[3].data_ptr(), geom,
                             ctx.act, part.data_ptr(), _native.stream(y), [y.numel(), dp.numel(), part.numel()])
        else:
            K.pool_bwd(dp.data_ptr(), y.data_ptr(), dz.data_ptr(), prm[2].data_ptr(), prm[3].data_ptr(), geom,
                       int(ctx.is_max), int(ctx.count_pad), ctx.act, _native.stream(y), [y.numel(), dp.numel()])
        y2, dz2 = y.reshape(-1, C), dz.reshape(-1, C)
        dbeta = dgamma = None
        if ctx.training or ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            dbeta, dgamma = _bwd_param_grads(dz2, y2, prm, ctx.act, *ctx.params, part=part)
        dy = _bwd_input(dz2, y2, prm, dbeta, dgamma, ctx.act, ctx.training) if ctx.needs_input_grad[0] else None
        return (None if dy is None else dy.reshape(y.shape), dgamma if ctx.has_gamma else None,
                dbeta if ctx.has_beta else None) + (None,) * 10


def batchnorm_act(y5, gamma, beta, running_mean, running_var, training: bool, momentum: float = 0.1,
                  eps: float = 1e-5, act=None, stats_slab=None, conv_next: bool = False):
    """z = act(bn(y)).  ``conv_next``: the caller promises that z goes to one ``ops.conv`` and
    nowhere else -- z may then be written by that conv's forward kernel (ops/bnfuse.py defer)."""
    if _native.use_native(y5):
        # (grad mode is off inside Function.forward: decide here whether a backward will run)
        tag = training and torch.is_grad_enabled() and (y5.requires_grad or any(
            p is not None and p.requires_grad for p in (gamma, beta)))
        return BatchNormActFn.apply(y5.to(torch.bfloat16).contiguous(), gamma, beta, stats_slab, running_mean,
                                    running_var, training, momentum, eps, act_code(act), tag, bool(conv_next))
    return ref.batchnorm_act(y5, gamma, beta, running_mean, running_var, training, momentum, eps, act)


def batchnorm_act_pool(y5, gamma, beta, running_mean, running_var, training: bool, pspec: PoolSpec,
                       kind: str = "max", momentum: float = 0.1, eps: float = 1e-5, act=None, stats_slab=None,
                       count_pad: bool = False):
    if _native.use_native(y5):
        return BatchNormActPoolFn.apply(y5.to(torch.bfloat16).contiguous(), gamma, beta, stats_slab, running_mean,
                                        running_var, training, momentum, eps, act_code(act), pspec, kind == "max",
                                        count_pad)
    z = ref.batchnorm_act(y5, gamma, beta, running_mean, running_var, training, momentum, eps, act)
    return ref.pool(z, pspec, kind, count_pad)


class BatchNormActPointwiseFn(torch.autograd.Function):
    """out = act(bn(y)) @ W^T + b for a 1x1x1 conv head: the pointwise kernels apply BN + act
    to their input tile in registers (forward and weight gradient), so act(bn(y)) -- the
    segmentation decoder's 64^3 x 32 output -- is never written or re-read.  Backward: the
    head's dgrad gives dz straight from dout, then the usual BN backward on (dz, y)."""

    @staticmethod
    def forward(ctx, y, gamma, beta, slab, rmean, rvar, momentum, eps, act, w, b):
        from .conv import pw_fwd

        C = y.shape[-1]
        y2 = y.reshape(-1, C)
        if slab is None:
            slab = _stats_slab(y2)
        prm = _finalize_fwd(slab, y2.shape[0], gamma, beta, rmean, rvar, momentum, eps)
        N = w.shape[0]
        w2 = w.detach().reshape(N, C)
        bias = b.detach().float().contiguous() if b is not None else None
        out = pw_fwd(y2, w2, bias, 0, pro=(prm[2], prm[3], act))
        ctx.save_for_backward(y, prm, w)
        ctx.act, ctx.has_b, ctx.bparam = act, b is not None, b
        ctx.params = (beta, gamma)
        return out.reshape(*y.shape[:-1], N)

    @staticmethod
    def backward(ctx, dout):
        from .conv import native_colsum, pw_fwd, pw_wgrad

        y, prm, w = ctx.saved_tensors
        C = y.shape[-1]
        N = w.shape[0]
        y2 = y.reshape(-1, C)
        d2 = dout.contiguous().to(torch.bfloat16).reshape(-1, N)
        w2 = w.detach().reshape(N, C)
        dw = (pw_wgrad(d2, y2, pro=(prm[2], prm[3], ctx.act), out=grad_target(w)).reshape(w.shape)
              if ctx.needs_input_grad[9] else None)
        db = native_colsum(d2, out=grad_target(ctx.bparam)) if (ctx.has_b and ctx.needs_input_grad[10]) else None
        M = y2.shape[0]
        Kn = _native.kernels()
        part = None
        if C <= 32 and N <= 32 and C % 8 == 0 and 2048 % C == 0:
            # d(act(bn(y))) [M, C] and this BN's raw backward moments in the same pass
            part = torch.empty(Kn.pw_fwd_blocks(M, N, C), 2, C, dtype=torch.float32, device=y.device)
            dz2 = torch.empty(M, C, dtype=torch.bfloat16, device=y.device)
            wb = w2.t().to(torch.bfloat16).contiguous()
            Kn.pw_fwd(d2.data_ptr(), wb.data_ptr(), 0, dz2.data_ptr(), M, N, C, 0, _native.stream(d2), 0, 0, 0,
                      y2.data_ptr(), prm[2].data_ptr(), prm[3].data_ptr(), part.data_ptr(), ctx.act)
        else:
            dz2 = pw_fwd(d2, w2.t(), None, 0)                # d(act(bn(y))) [M, C]
        dbeta, dgamma = _bwd_param_grads(dz2, y2, prm, ctx.act, *ctx.params, part=part)
        dy = _bwd_input(dz2, y2, prm, dbeta, dgamma, ctx.act, True) if ctx.needs_input_grad[0] else None
        return (None if dy is None else dy.reshape(y.shape), dgamma if ctx.needs_input_grad[1] else None,
                dbeta if ctx.needs_input_grad[2] else None, None, None, None, None, None, None, dw, db)


def batchnorm_act_pointwise(y5, gamma, beta, running_mean, running_var, w, b, momentum: float = 0.1,
                            eps: float = 1e-5, act=None, stats_slab=None):
    """Training-mode ``conv1x1(act(bn(y)))`` with the BN + act inside the 1x1 conv's kernels
    (GPU; the caller checks :func:`fused_pointwise_ok`)."""
    return BatchNormActPointwiseFn.apply(y5.to(torch.bfloat16).contiguous(), gamma, beta, stats_slab, running_mean,
                                         running_var, momentum, eps, act_code(act), w, b)


def fused_pointwise_ok(y5, C: int, N: int, act) -> bool:
    from .conv import pw_prologue_ok

    import os

    M = y5.numel() // C
    return (os.environ.get("FN_BN_PW_FUSE", "1") != "0" and _native.use_native(y5) and pw_prologue_ok(C)
            and C <= 64 and N <= 64 and M % 8 == 0 and act in (None, "relu"))
