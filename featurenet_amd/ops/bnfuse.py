"""Cross-op fusion of a BN layer's backward statistics into the next conv's dgrad.

A FeatureNet-3D block is ``conv -> BN -> act`` and the next block's conv reads
``z = act(bn(y))``.  In backward that conv's dgrad writes ``dz``, and the BN
backward then needs ``sum g`` and ``sum g * xhat`` (``g = dz * act'(z)``): one
full pass over ``dz`` and ``y`` (``colstats``).  Instead the BN forward writes its relu
mask, the big-tile dgrad's epilogue sums ``g`` from registers (its loader DMAs the mask
bytes), and ``sum g * xhat`` follows from the adjoint identity ``sum_p dz z = sum W . dW``
over the conv's weights and weight gradient (:func:`identity_ok`), so the pass disappears.

Autograd runs the two ops as separate Functions, so they meet here:

* :func:`tag_output` -- BN forward records ``z -> (y, prm, act, mask)``;
* :func:`source_of` -- the consuming conv's forward looks its input up;
* :func:`offer` -- its backward hands ``(dz, ("identity", sum-g slab, S partials))`` over;
* :func:`take` -- the BN backward claims the slab for its ``dz`` (else it runs
  ``colstats`` as before).

Entries hold weak references and are matched on storage pointer, numel, the
identity of ``y`` and the version counter of ``dz``: when the BN output has
other consumers, autograd may add their gradients into the conv's ``dx`` in
place (same storage, bumped version), and the slab then describes only the
conv branch -- the version check turns that into a miss.  A miss (a fork in the
graph, the halo kernel chosen for dgrad, no-grad forward) only falls back to the
separate pass.
"""
from __future__ import annotations

import os
import threading
import weakref

import torch

_LOCK = threading.Lock()
_FWD: dict = {}      # z.data_ptr() -> (ref z, ref y, ref prm, act)
_BWD: dict = {}      # dz.data_ptr() -> (ref dz, slab, ref y, dz._version at offer)


def identity_enabled() -> bool:
    """BN backward without the colstats pass (``FN_BN_IDENTITY``, default on): the BN forward
    writes its relu mask, the consuming conv's 16x16x32 tile dgrad stores g = dz * mask and its
    column sums, and ``sum g * xhat`` comes from the adjoint identity
    ``sum_p dz z = sum W * dW`` over the conv's weights and weight gradient
    (``bn_pool.hip`` bn_bwd_prep_kernel)."""
    return os.environ.get("FN_BN_IDENTITY", "1") != "0"


def identity_ok(C: int, act: int) -> bool:
    """The identity path's shape conditions: relu (the mask) and 32 or 64 channels (one or two
    mask dwords per position for the dgrad loader's DMA)."""
    return identity_enabled() and act == 1 and C in (32, 64)


def pool_stats_enabled() -> bool:
    """BN-backward moments inside the max-pool backward (FN_POOL_BN_STATS, default on)."""
    return os.environ.get("FN_POOL_BN_STATS", "1") != "0"


def pool_apply_enabled() -> bool:
    """BN backward's input gradient computed inside the max-pool backward (the moments pass then
    writes nothing; ``pool_bn_bwd_apply``) -- FN_POOL_BN_APPLY, default on."""
    return os.environ.get("FN_POOL_BN_APPLY", "1") != "0"


def _purge(d: dict, limit: int = 256) -> None:
    if len(d) > limit:
        for k in [k for k, v in d.items() if v[0]() is None]:
            d.pop(k, None)


def tag_output(z: torch.Tensor, y: torch.Tensor, prm: torch.Tensor, act: int, mask=None) -> None:
    """BN forward (training): z = act(y * prm[2] + prm[3]), prm = (mean, invstd, scale, shift);
    ``mask``: z's relu-mask bytes (the identity path; the BN keeps it alive until its backward)."""
    if mask is None:
        return
    with _LOCK:
        _purge(_FWD)
        _FWD[z.data_ptr()] = (weakref.ref(z), weakref.ref(y), weakref.ref(prm), act,
                              weakref.ref(mask) if mask is not None else None)


def source_of(x: torch.Tensor):
    """(y, prm, act, mask) when ``x`` is (a same-extent view of) a tagged BN output, else None
    (mask: the relu-mask bytes, or None)."""
    e = _FWD.get(x.data_ptr())
    if e is None:
        return None
    z, y, prm = e[0](), e[1](), e[2]()
    if z is None or y is None or prm is None or z.numel() != x.numel() or not x.is_contiguous():
        return None
    mask = e[4]() if e[4] is not None else None
    return y, prm, e[3], mask


_LAZY: dict = {}     # z.data_ptr() -> (ref z, y, prm, act, mask, fill)


def prologue_enabled() -> bool:
    """BN + relu of a conv's input inside the consuming conv_tile forward (``FN_BN_PROLOGUE=1``;
    off by default): the BN forward leaves ``z`` unwritten, the conv's loader normalises the landed
    halo of ``y`` in LDS and writes ``z`` (and the relu mask) once, for the positions its tile owns
    (conv_tile.hip ``xform_job``) -- no ``bn_apply`` pass.  Bit-identical, but measured slower:
    the loader shares SIMD 0 with compute wave 0, and its ~20 VALU instructions per 16-B chunk
    take MFMA issue cycles from that wave -- the forward convs ran 1.6-2.3x longer, far more than
    the 170 us of bn_apply passes they replace (profiles/r6_bn_prologue.md)."""
    return os.environ.get("FN_BN_PROLOGUE", "0") == "1"


def prologue_wgrad_enabled() -> bool:
    """The weight gradient of the conv that took a BN prologue normalises its x halos itself
    (``FN_BN_PROLOGUE_WGRAD=1``) instead of reading the z that the forward's loader writes
    (default): the loader has idle cycles for the write, the weight-gradient waves have none for
    the normalisation."""
    return os.environ.get("FN_BN_PROLOGUE_WGRAD", "0") == "1"


def defer(z: torch.Tensor, y: torch.Tensor, prm: torch.Tensor, act: int, mask, fill) -> None:
    """BN forward with a promised conv consumer: ``z`` is allocated but not written; ``fill()``
    writes it (and ``mask``) with the separate pass if the consumer cannot take the prologue."""
    with _LOCK:
        _purge(_LAZY)
        _LAZY[z.data_ptr()] = (weakref.ref(z), y, prm, act, mask, fill)


def pending(x: torch.Tensor):
    """(y, prm, act, mask) when ``x`` is a deferred BN output not yet written, else None."""
    e = _LAZY.get(x.data_ptr())
    if e is None or e[0]() is None or e[0]().numel() != x.numel():
        return None
    return e[1], e[2], e[3], e[4]


def filler(x: torch.Tensor):
    """The separate pass that writes the deferred ``x`` (and its mask), for a later reader."""
    e = _LAZY.get(x.data_ptr())
    return e[5] if e is not None else (lambda: None)


def settle(x: torch.Tensor, written: bool) -> None:
    """The deferred ``x`` is dealt with: ``written`` -- the consumer's prologue wrote z and the mask;
    otherwise the separate pass writes them now (before anything reads ``x``)."""
    with _LOCK:
        e = _LAZY.pop(x.data_ptr(), None)
    if e is not None and not written:
        e[5]()


def offer(dz: torch.Tensor, slab, y: torch.Tensor) -> None:
    """``slab``: ``("identity", gslab, wpart)`` -- the tile dgrad's sum-g slab and the S partials of
    the conv's W . dW."""
    with _LOCK:
        _purge(_BWD)
        _BWD[dz.data_ptr()] = (weakref.ref(dz), slab, weakref.ref(y), dz._version)


def take(dz: torch.Tensor, y: torch.Tensor):
    """What :func:`offer` handed over for this (dz, y) pair, or None."""
    with _LOCK:
        e = _BWD.pop(dz.data_ptr(), None)
    if e is None:
        return None
    d, yy = e[0](), e[2]()
    if d is None or yy is None or d.numel() != dz.numel() or yy.data_ptr() != y.data_ptr():
        return None
    if dz._version != e[3] or d._version != e[3]:
        return None                               # modified since (another branch's gradient added)
    return e[1]
