"""Dense layer: ``y = act(x @ W^T + b)``.

Reference parity: Keras ``Dense`` (``model/input.py:174-190``) and the
classifier head ``Dense(n_classes, softmax)`` (``model/keras_model.py:124``).

GPU: hand-written MFMA kernels (``csrc/kernels/dense.hip``): split-K forward
that reads the fp32 master weights directly (no per-step bf16 weight copy) with
bias + activation in the split reduction, a dgrad and a weight-gradient kernel
that writes the fp32 ``dW`` (and ``db``) straight into the parameters' flat
gradients.  Any K / N / M: the kernels pad the MFMA dims with zeros and load unaligned rows
element-wise; the weight gradient splits the batch into slices (own dW slabs, summed in a
fixed order) so small dW matrices still fill the GPU.  A softmax activation (a Dense inside a
NAS candidate) is a native row-softmax kernel with its own backward (``misc.hip``).  torch /
hipBLASLt only with ``FN_DENSE_NATIVE=0`` (the A/B switch).
"""
from __future__ import annotations

import os

import torch

from .. import _native
from ..training.flat import grad_target
from . import reference as ref
from .spec import act_code

_NATIVE = os.environ.get("FN_DENSE_NATIVE", "1") != "0"


def _torch_fwd(xb: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    return torch.matmul(xb, w.detach().to(torch.bfloat16).t())


def _wgrad_torch(dy2: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
    """fp32 dW = dy^T x straight out of the GEMM (no bf16 round trip, no cast pass)."""
    try:
        return torch.mm(dy2.t(), x2, out_dtype=torch.float32)
    except (TypeError, RuntimeError):
        return torch.matmul(dy2.t(), x2).float()


class LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act: int, out_fp32: bool):
        K = x.shape[-1]
        N = w.shape[0]
        x2 = x.reshape(-1, K).to(torch.bfloat16).contiguous()
        M = x2.shape[0]
        wf = w.detach()
        bias = b.detach().float().contiguous() if b is not None else None
        native = _NATIVE and wf.dtype == torch.float32 and wf.is_contiguous()
        if native:
            Kn = _native.kernels()
            S = int(Kn.dense_splits(M, N, K))
            part = torch.empty(S, M, N, dtype=torch.float32, device=x.device)
            y = torch.empty(M, N, dtype=torch.float32 if out_fp32 else torch.bfloat16, device=x.device)
            Kn.dense_fwd(x2.data_ptr(), wf.data_ptr(), _native.ptr(bias), y.data_ptr(), part.data_ptr(), M, N, K, S,
                         act, int(out_fp32), _native.stream(x2), [x2.numel(), wf.numel(), y.numel(), part.numel()])
        else:
            y = _torch_fwd(x2, wf)
            if b is not None or act:
                y2 = torch.empty_like(y)
                _native.kernels().bias_act(y.data_ptr(), _native.ptr(bias), y2.data_ptr(), y.numel(), N, act,
                                           _native.stream(y))
                y = y2
            if out_fp32:
                y = y.float()
        ctx.save_for_backward(x2, w, y if act else None)
        ctx.act, ctx.has_b, ctx.xshape = act, b is not None, x.shape
        ctx.bparam = b
        return y.reshape(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, w, y = ctx.saved_tensors
        M, K = x2.shape
        N = w.shape[0]
        g = dy.reshape(M, N).to(torch.bfloat16).contiguous()
        wf = w.detach()
        NP = -(-N // 32) * 32                          # (any N: the dgrad kernel pads its k dim to 32)
        # (any K: the kernel stages W rows and stores dx rows that are not 16-B aligned element by element)
        dgrad_native = _NATIVE and wf.dtype == torch.float32 and 64 * (NP + 8) * 2 <= 160 * 1024
        # the activation backward inside the dgrad / wgrad kernels (g = dy * act'(y) as they load
        # it) when both run natively and the wgrad kernel produces db: no separate pass.  Small
        # layers only (K <= 4096): every dgrad / wgrad workgroup re-applies it to the g rows it
        # reads, which for FC1 (K = 64000: 1000 column workgroups) cost more than the pass
        ya = None
        if ctx.act:
            if (_NATIVE and K <= 4096 and ctx.needs_input_grad[1] and (dgrad_native or not ctx.needs_input_grad[0])
                    and y.dtype == torch.bfloat16):
                ya = y.reshape(M, N).contiguous()
            else:
                g2 = torch.empty_like(g)
                _native.kernels().act_bwd(g.data_ptr(), y.reshape(M, N).to(torch.bfloat16).contiguous().data_ptr(),
                                          g2.data_ptr(), g.numel(), ctx.act, _native.stream(g))
                g = g2
        yp, yact = (_native.ptr(ya), ctx.act) if ya is not None else (0, 0)
        Kn = _native.kernels()
        st = _native.stream(g)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            if dgrad_native:
                dx = torch.empty(M, K, dtype=torch.bfloat16, device=g.device)
                Kn.dense_dgrad(g.data_ptr(), wf.data_ptr(), dx.data_ptr(), M, N, K, st,
                               [g.numel(), wf.numel(), dx.numel()] + ([ya.numel()] if ya is not None else []), yp,
                               yact)
            else:
                dx = torch.matmul(g, wf.to(torch.bfloat16))
            dx = dx.reshape(ctx.xshape)
        want_b = ctx.has_b and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1]:
            if _NATIVE:                                # (batch slices fill the GPU for small dW)
                dw = grad_target(w)
                if dw is None:
                    dw = torch.empty(N, K, dtype=torch.float32, device=g.device)
                if want_b:
                    db = grad_target(ctx.bparam)
                    if db is None:
                        db = torch.empty(N, dtype=torch.float32, device=g.device)
                S = int(Kn.dense_wgrad_slices(M, N, K))
                part = torch.empty(S * (N * K + N), dtype=torch.float32, device=g.device) if S > 1 else None
                Kn.dense_wgrad(g.data_ptr(), x2.data_ptr(), dw.data_ptr(), _native.ptr(db), M, N, K, st,
                               [g.numel(), x2.numel(), dw.numel(), part.numel() if S > 1 else 0,
                                ya.numel() if ya is not None else 0], _native.ptr(part), S, yp, yact)
            else:
                dw = _wgrad_torch(g, x2)
        if want_b and db is None:
            db = g.float().sum(0)
        return dx, dw, db, None, None


@torch.no_grad()
def linear_infer(x: torch.Tensor, w_bf16: torch.Tensor, b: torch.Tensor | None = None, act=None,
                 out_fp32: bool = False) -> torch.Tensor:
    """Inference forward with a bf16 weight copy (half the weight bytes of the fp32 master
    weights, no conversion in the loop): FC1 of the 128^3 inference config reads a 1024 x
    1.1M bf16 activation against a 128 x 1.1M weight.  Native kernel only (no autograd)."""
    K = x.shape[-1]
    N = w_bf16.shape[0]
    if w_bf16.dtype != torch.bfloat16 or not w_bf16.is_contiguous() or w_bf16.shape[1] != K:
        raise ValueError("linear_infer: w_bf16 must be a contiguous bf16 [N, K] tensor")
    x2 = x.reshape(-1, K).to(torch.bfloat16).contiguous()
    M = x2.shape[0]
    bias = b.detach().float().contiguous() if b is not None else None
    Kn = _native.kernels()
    S = int(Kn.dense_splits(M, N, K))
    part = torch.empty(S, M, N, dtype=torch.float32, device=x.device)
    y = torch.empty(M, N, dtype=torch.float32 if out_fp32 else torch.bfloat16, device=x.device)
    Kn.dense_fwd(x2.data_ptr(), w_bf16.data_ptr(), _native.ptr(bias), y.data_ptr(), part.data_ptr(), M, N, K, S,
                 act_code(act), int(out_fp32), _native.stream(x2), [x2.numel(), w_bf16.numel(), y.numel(),
                                                                     part.numel()], 1)
    return y.reshape(*x.shape[:-1], N)


class SoftmaxRowsFn(torch.autograd.Function):
    """softmax over the last axis of an fp32 tensor on the native row kernels (forward and backward)."""

    @staticmethod
    def forward(ctx, x):
        N = x.shape[-1]
        x2 = x.reshape(-1, N).contiguous()
        y = torch.empty_like(x2)
        _native.kernels().softmax_rows(x2.data_ptr(), y.data_ptr(), x2.shape[0], N, 0, 0, _native.stream(x2),
                                       [x2.numel(), y.numel()])
        ctx.save_for_backward(y)
        return y.reshape(x.shape)

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        N = y.shape[-1]
        g2 = g.reshape(-1, N).float().contiguous()
        dx = torch.empty_like(y)
        _native.kernels().softmax_rows(y.data_ptr(), dx.data_ptr(), y.shape[0], N, 1, g2.data_ptr(),
                                       _native.stream(y), [y.numel(), dx.numel(), g2.numel()])
        return dx.reshape(g.shape)


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None, act=None, out_fp32: bool = False):
    if _native.use_native(x):
        if act == "softmax":
            y = LinearFn.apply(x, w, b, 0, True)
            return SoftmaxRowsFn.apply(y)
        return LinearFn.apply(x, w, b, act_code(act), out_fp32)
    y = torch.nn.functional.linear(x, w.to(x.dtype), None if b is None else b.to(x.dtype))
    return ref.activation(y, act)
