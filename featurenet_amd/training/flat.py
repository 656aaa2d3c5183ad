"""Flat parameter / gradient storage.

Every trainable parameter of a model is re-pointed into ONE fp32 buffer and
its ``.grad`` into ONE matching fp32 gradient buffer.  Layout is *reverse
registration order*, i.e. the order in which backward produces gradients, so
data-parallel gradient buckets are contiguous slices that become ready one
after the other (see :mod:`featurenet_amd.parallel.ddp`).  The optimizer
(:mod:`featurenet_amd.ops.optim`) then updates the whole model in a single
kernel launch.

Direct gradients: ``zero_grad`` clears the flat gradient and sets every
``p.grad`` to ``None``; a backward that can write a parameter's gradient in
place asks :func:`grad_target` for the parameter's (zeroed) flat slice, writes
it and returns that slice, which autograd then adopts as ``p.grad`` without a
copy or an accumulate kernel.  Any other gradient is copied into the flat slice
by a post-accumulate hook, so the flat buffer always holds every gradient.
"""
from __future__ import annotations

import weakref

import torch
from torch import nn

ALIGN = 64  # elements (256 B): every slice starts on a 256-byte boundary

# parameter data pointer -> (FlatParams, parameter, flat gradient view)
_DIRECT: "weakref.WeakValueDictionary[int, _Slot]" = weakref.WeakValueDictionary()


class _Slot:
    __slots__ = ("flat", "param", "view", "claimed", "__weakref__")

    def __init__(self, flat, param, view):
        self.flat, self.param, self.view, self.claimed = flat, param, view, False


def grad_target(p: torch.Tensor):
    """The zeroed flat gradient slice of parameter ``p`` (shape of ``p``) when the current
    backward may write ``p``'s gradient there directly, else ``None``.  At most once per
    step per parameter (a parameter used twice gets its second gradient accumulated by
    autograd as usual)."""
    if p is None:
        return None
    slot = _DIRECT.get(p.data_ptr())
    if slot is None or slot.claimed or slot.param.grad is not None or slot.view.shape != p.shape:
        return None
    slot.claimed = True
    return slot.view.view(slot.view.shape)   # a fresh alias: autograd adopts it without a copy


def _adopt_hook(p) -> None:
    """Post-accumulate-grad hook of every flat parameter: a module-level function (not a
    bound method), so a hook left on a parameter never keeps a FlatParams alive."""
    slot = _DIRECT.get(p.data_ptr())
    if slot is not None and slot.flat is not None:
        slot.flat._adopt(p)


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
        self._slots = []
        self._hooks = []
        # a FlatParams built again on the same parameters supersedes the old one: drop the
        # old hooks (they would pile up and keep its buffers alive through the bound method)
        for p in params:
            old = _DIRECT.get(p.data_ptr())
            if old is not None and old.flat is not None:
                old.flat.release()
        with torch.no_grad():
            for p, off in zip(params, offs):
                n = p.numel()
                self.data[off:off + n].copy_(p.detach().reshape(-1).float())
                p.data = self.data[off:off + n].view(p.shape)
                view = self.grad[off:off + n].view(p.shape)
                p.grad = view
                self.slices.append((p, off, n))
                slot = _Slot(self, p, view)
                self._slots.append(slot)
                _DIRECT[p.data_ptr()] = slot
                self._hooks.append(p.register_post_accumulate_grad_hook(_adopt_hook))
        self.module = module

    def release(self) -> None:
        """Detach this FlatParams from its parameters' gradient hooks and direct-gradient
        slots (the parameters keep pointing into ``data``)."""
        for h in self._hooks:
            h.remove()
        self._hooks = []
        for slot in self._slots:
            if _DIRECT.get(slot.param.data_ptr()) is slot:
                del _DIRECT[slot.param.data_ptr()]
            slot.flat = None
        self._slots = []

    @property
    def n_params(self) -> int:
        return sum(n for _, _, n in self.slices)

    def zero_grad(self) -> None:
        self.grad.zero_()
        for slot in self._slots:
            slot.param.grad = None
            slot.claimed = False

    def _adopt(self, p) -> None:  # noqa: D401 - see _adopt_hook
        """Post-accumulate hook: make ``p.grad`` the flat slice (copying a gradient autograd
        produced elsewhere).  Runs before any data-parallel bucket hook of ``p``."""
        slot = _DIRECT.get(p.data_ptr())
        if slot is None or slot.flat is not self or p.grad is None:
            return
        if p.grad.data_ptr() != slot.view.data_ptr():
            with torch.no_grad():
                slot.view.copy_(p.grad)
            p.grad = slot.view

    def check_bound(self) -> None:
        """Raise if a parameter was re-bound away from the flat buffer (e.g. ``module.to``)."""
        for p, off, n in self.slices:
            if p.data_ptr() != self.data[off:off + n].data_ptr():
                raise RuntimeError("parameter detached from FlatParams storage; rebuild FlatParams after .to()")
