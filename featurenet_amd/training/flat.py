"""Flat parameter / gradient storage.

Every trainable parameter of a model is re-pointed into ONE fp32 buffer and
its ``.grad`` into ONE matching fp32 gradient buffer.  Layout is *reverse
registration order*, i.e. the order in which backward produces gradients, so
data-parallel gradient buckets are contiguous slices that become ready one
after the other (see :mod:`featurenet_amd.parallel.ddp`).  The optimizer
(:mod:`featurenet_amd.ops.optim`) then updates the whole model in a single
kernel launch.
"""
from __future__ import annotations

import torch
from torch import nn

ALIGN = 64  # elements (256 B): every slice starts on a 256-byte boundary


class FlatParams:
    def __init__(self, module: nn.Module, order: str = "reverse"):
        params = [p for p in module.parameters() if p.requires_grad]
        if order == "reverse":
            params = params[::-1]
        if not params:
            raise ValueError("module has no trainable parameters")
        device = params[0].device
        offs, total = [], 0
        for p in params:
            offs.append(total)
            total += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.numel = total
        self.data = torch.zeros(total, dtype=torch.float32, device=device)
        self.grad = torch.zeros(total, dtype=torch.float32, device=device)
        self.slices: list[tuple[nn.Parameter, int, int]] = []
        with torch.no_grad():
            for p, off in zip(params, offs):
                n = p.numel()
                self.data[off:off + n].copy_(p.detach().reshape(-1).float())
                p.data = self.data[off:off + n].view(p.shape)
                p.grad = self.grad[off:off + n].view(p.shape)
                self.slices.append((p, off, n))
        self.module = module

    @property
    def n_params(self) -> int:
        return sum(n for _, _, n in self.slices)

    def zero_grad(self) -> None:
        self.grad.zero_()

    def check_bound(self) -> None:
        """Raise if a parameter was re-bound away from the flat buffer (e.g. ``module.to``)."""
        for p, off, n in self.slices:
            if p.data_ptr() != self.data[off:off + n].data_ptr():
                raise RuntimeError("parameter detached from FlatParams storage; rebuild FlatParams after .to()")
