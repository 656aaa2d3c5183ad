"""Flat-buffer optimizers (Adam / SGD) backed by one fused HIP kernel each.

All trainable parameters of a model live in ONE fp32 allocation
(:class:`featurenet_amd.training.flat.FlatParams`), so an optimizer step is a
single kernel launch over the whole buffer regardless of how many layers the
NAS candidate has, and the data-parallel all-reduce can work on contiguous
slices of the matching flat gradient buffer.

Reference parity: ``Adam(lr=1e-3)`` (``tensorflow_generator.py:232``) with
Keras 2.2's epsilon placement (``keras_eps=True``), and the SGD used by the
hand-written baselines (``lenet5.py``).
"""
from __future__ import annotations

import math

import torch

from .. import _native


class FlatAdam:
    def __init__(self, params: torch.Tensor, grads: torch.Tensor, lr: float = 1e-3, betas=(0.9, 0.999),
                 eps: float = 1e-7, weight_decay: float = 0.0, keras_eps: bool = True, shadow: torch.Tensor | None = None):
        assert params.dtype == torch.float32 and params.is_contiguous()
        self.p, self.g = params, grads
        self.m = torch.zeros_like(params)
        self.v = torch.zeros_like(params)
        self.lr, self.b1, self.b2, self.eps, self.wd = lr, betas[0], betas[1], eps, weight_decay
        self.keras_eps = keras_eps
        self.shadow = shadow
        self.t = 0
        self._dev = None     # (hp, t) device state of the graph-capturable form
        self._gscale = 1.0   # gradient scale of the device state (1/world under data parallelism)
        self._pushed = None  # the host hyper-parameters last copied to the device state

    # ------------------------------------------------------------ graph mode
    def enable_device_state(self, grad_scale: float | None = None) -> None:
        """Keep lr / betas / step / gradient scale on the device so a captured step replays
        correctly."""
        if grad_scale is not None:
            self._gscale = float(grad_scale)
        if self._dev is None:
            hp = torch.tensor([self.lr, self.b1, self.b2, self.eps, self.wd, self._gscale], dtype=torch.float32,
                              device=self.p.device)
            t = torch.tensor([self.t], dtype=torch.int32, device=self.p.device)
            self._dev = (hp, t)
            self._pushed = self._host_hp()
        else:
            self.sync_device_state()

    def sync_device_state(self, grad_scale: float | None = None) -> None:
        """Push host-side hyper-parameter changes (e.g. an lr callback) to the device copy
        (``grad_scale`` None keeps the current one)."""
        if grad_scale is not None:
            self._gscale = float(grad_scale)
        if self._dev is not None:
            self._pushed = self._host_hp()
            self._dev[0].copy_(torch.tensor(list(self._pushed)))

    def _host_hp(self) -> tuple:
        return (float(self.lr), float(self.b1), float(self.b2), float(self.eps), float(self.wd), float(self._gscale))

    def step_device(self) -> None:
        """One Adam step entirely driven by device state (safe inside hipGraph capture)."""
        hp, t = self._dev
        _native.kernels().adam_flat_dev(self.p.data_ptr(), self.g.data_ptr(), self.m.data_ptr(), self.v.data_ptr(),
                                        _native.ptr(self.shadow), self.p.numel(), hp.data_ptr(), t.data_ptr(),
                                        int(self.keras_eps), _native.stream(self.p))

    def step(self, grad_scale: float = 1.0) -> None:
        if self._dev is not None and _native.use_native(self.p):
            # eager steps with the device state (e.g. after a graph-capture fallback): push any
            # host-side change -- a new lr from a callback, another gradient scale -- first
            if grad_scale != self._gscale or self._host_hp() != self._pushed:
                self.sync_device_state(grad_scale)
            self.t += 1
            self.step_device()
            return
        self.t += 1
        bc1 = 1.0 - self.b1 ** self.t
        bc2 = 1.0 - self.b2 ** self.t
        if _native.use_native(self.p):
            _native.kernels().adam_flat(self.p.data_ptr(), self.g.data_ptr(), self.m.data_ptr(), self.v.data_ptr(),
                                        _native.ptr(self.shadow), self.p.numel(), self.lr, self.b1, self.b2, self.eps,
                                        self.wd, bc1, bc2, grad_scale, int(self.keras_eps), _native.stream(self.p))
            return
        with torch.no_grad():
            g = self.g * grad_scale
            self.m.mul_(self.b1).add_(g, alpha=1 - self.b1)
            self.v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            if self.wd:
                self.p.mul_(1 - self.lr * self.wd)
            if self.keras_eps:
                lr_t = self.lr * math.sqrt(bc2) / bc1
                self.p.addcdiv_(self.m, self.v.sqrt().add_(self.eps), value=-lr_t)
            else:
                denom = (self.v / bc2).sqrt_().add_(self.eps)
                self.p.addcdiv_(self.m / bc1, denom, value=-self.lr)
            if self.shadow is not None:
                self.shadow.copy_(self.p)

    def state_dict(self) -> dict:
        return {"m": self.m, "v": self.v, "t": self.t, "lr": self.lr, "betas": (self.b1, self.b2), "eps": self.eps,
                "weight_decay": self.wd, "keras_eps": self.keras_eps}

    def load_state_dict(self, sd: dict) -> None:
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self.t = int(sd["t"])
        self.lr = float(sd.get("lr", self.lr))
        if self._dev is not None:
            self._dev[1].fill_(self.t)
            self.sync_device_state()


class FlatSGD:
    def __init__(self, params: torch.Tensor, grads: torch.Tensor, lr: float = 0.01, momentum: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, shadow: torch.Tensor | None = None):
        self.p, self.g = params, grads
        self.buf = torch.zeros_like(params)
        self.lr, self.momentum, self.wd, self.nesterov = lr, momentum, weight_decay, nesterov
        self.shadow = shadow
        self.t = 0

    def step(self, grad_scale: float = 1.0) -> None:
        self.t += 1
        if _native.use_native(self.p):
            _native.kernels().sgd_flat(self.p.data_ptr(), self.g.data_ptr(), self.buf.data_ptr(),
                                       _native.ptr(self.shadow), self.p.numel(), self.lr, self.momentum, self.wd,
                                       int(self.nesterov), grad_scale, _native.stream(self.p))
            return
        with torch.no_grad():
            g = self.g * grad_scale
            if self.wd:
                g = g + self.wd * self.p
            if self.momentum:
                self.buf.mul_(self.momentum).add_(g)
                g = g + self.momentum * self.buf if self.nesterov else self.buf
            self.p.add_(g, alpha=-self.lr)
            if self.shadow is not None:
                self.shadow.copy_(self.p)

    def state_dict(self) -> dict:
        return {"buf": self.buf, "t": self.t, "lr": self.lr, "momentum": self.momentum}

    def load_state_dict(self, sd: dict) -> None:
        self.buf.copy_(sd["buf"])
        self.t = int(sd["t"])
        self.lr = float(sd.get("lr", self.lr))
