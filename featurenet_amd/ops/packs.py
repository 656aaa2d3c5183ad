"""A model forward's weight packs in one launch.

Every conv re-packs its fp32 master weights into its kernel's bf16 B-operand layout each step
(the weights move every optimizer step): the gather (igemm) and halo layouts of NAS candidates,
the tile-kernel streams of FeatureNet-3D (forward + dgrad in one launch per layer).  Each pack
is a 3-6 us launch -- ~4 of a LeNet candidate step's ~43 kernels, 3 of the FeatureNet-3D step's.

A model forward run in a :class:`pack_scope` makes every pack its layers made before --
recorded the first time each one missed -- in ONE ``pack_w_multi`` launch up front
(``csrc/kernels/pack_w.h``: one element map per layout kind, <= 24 jobs per launch); the layers,
and their backward (the autograd nodes keep the forward's generation and run under
:class:`gen_as`), take the packed operands from that generation's cache.  A generation's cache
is dropped when the model's next scope opens, so a pack never outlives the weights it was made
from (the optimizer step comes between two forwards), and the cache is owned by the model (a
weak map finds it by generation): a dropped NAS candidate takes its packs with it.

Layout kinds (the builders register themselves): 0-2 gather forward / dgrad / packed-W and 3 / 4
halo forward / dgrad (``ops/conv.py``), 5 tile-kernel stream (``ops/conv_tile.py``).  NAS
candidates (``ir/compile.py`` CandidateNet) run in a scope: 2.5 % off a LeNet step.  The
FeatureNet-3D models do not: their three tile-stream packs in one launch measured neutral.
"""
from __future__ import annotations

import os
import threading
import weakref

import torch

from .. import _native

MAXJ = 24                               # jobs per launch (csrc pack_w.h FN_PACK_MAXJ)
_LOCK = threading.Lock()
_NEXT = [0]
# kind -> (builder(p, desc, kind) -> (job row, output tensor, cache value), backward_only(desc, kind))
_BUILDERS: dict = {}


def register(kinds, builder, backward_only):
    for k in kinds:
        _BUILDERS[k] = (builder, backward_only)


class _PackGen:
    """One scope's packs: cache {key: packed}, the model's plan and its parameters by data
    pointer.  Held by the model (the current one only), reachable by generation number through
    a weak map."""
    __slots__ = ("cache", "plan", "params", "__weakref__")

    def __init__(self, plan, params):
        self.cache, self.plan, self.params = {}, plan, params


GENS = weakref.WeakValueDictionary()    # generation -> _PackGen


class _TLS(threading.local):
    gen = None                          # the generation this thread's pack calls belong to


TLS = _TLS()


def key(w: torch.Tensor, desc, kind: int):
    return (w.data_ptr(), tuple(w.shape), desc, kind)


def lookup(w: torch.Tensor, desc, kind: int):
    """The packed operand this scope's up-front launch made, or None -- also None when the
    parameter was changed in place since (its version counter moved: an EMA / SWA swap, a
    ``load_state_dict`` copy, a clamp between a forward and its backward), so the caller packs
    the current values instead of using a stale pack."""
    gen = TLS.gen
    g = GENS.get(gen) if gen is not None else None
    if g is None:
        return None
    hit = g.cache.get(key(w, desc, kind))
    if hit is None or hit[1] != w._version:
        return None
    return hit[0]


def record(w: torch.Tensor, desc, kind: int):
    """A pack made outside the cache: the scope's model makes it up front from now on (model
    parameters only -- fp32, contiguous; a per-step temporary is not recorded)."""
    gen = TLS.gen
    g = GENS.get(gen) if gen is not None else None
    if g is None:
        return
    p = g.params.get(w.data_ptr())
    if p is None or tuple(p.shape) != tuple(w.shape):
        return
    with _LOCK:
        g.plan.setdefault(key(w, desc, kind), (p, desc, kind))


class pack_scope:
    """``with pack_scope(model): y = <model body>`` -- the model's recorded weight packs in one
    launch at the start.  No-op on the CPU, without the native kernels or with
    ``FN_PACK_SCOPE=0`` (every layer packs its own weights: the A/B baseline)."""

    def __init__(self, model: torch.nn.Module):
        self.model = model
        self.prev = None

    def __enter__(self):
        m = self.model
        self.prev = TLS.gen
        plist = [p for p in m.parameters() if p.is_cuda]
        if not plist or not _native.kernels_available() or os.environ.get("FN_PACK_SCOPE", "1") == "0":
            TLS.gen = None
            return self
        params = {p.data_ptr(): p for p in plist if p.dtype == torch.float32 and p.is_contiguous()}
        plan = m.__dict__.setdefault("_pack_plan", {})
        g = _PackGen(plan, params)
        with _LOCK:
            _NEXT[0] += 1
            gen = _NEXT[0]
            GENS[gen] = g
        m.__dict__["_pack_gen"] = gen
        m.__dict__["_pack_gen_obj"] = g          # (the previous generation's packs go with it)
        jobs, ext = [], []
        grad = torch.is_grad_enabled()
        for k, (p, desc, kind) in list(plan.items()):
            if p.data_ptr() != k[0] or params.get(k[0]) is not p:
                plan.pop(k, None)                # (the parameter moved: re-recorded on its next miss)
                continue
            build, bwd_only = _BUILDERS[kind]
            if not grad and bwd_only(desc, kind):
                continue                         # (no backward under no_grad)
            row, out, val = build(p, desc, kind)
            jobs.append(row)
            ext.append((p.numel(), out.numel()))
            g.cache[k] = (val, p._version)       # (lookup checks the version: no stale packs)
        st = _native.stream(plist[0]) if jobs else None
        for i in range(0, len(jobs), MAXJ):
            _native.kernels().pack_w_multi([v for r in jobs[i:i + MAXJ] for v in r], st,
                                           [v for e in ext[i:i + MAXJ] for v in e])
        TLS.gen = gen
        return self

    def __exit__(self, *exc):
        TLS.gen = self.prev
        return False


class gen_as:
    """The pack calls of a backward belong to its forward's generation (autograd runs the
    backward on another thread)."""

    def __init__(self, gen):
        self.gen = gen
        self.prev = None

    def __enter__(self):
        self.prev = TLS.gen
        TLS.gen = self.gen
        return self

    def __exit__(self, *exc):
        TLS.gen = self.prev
        return False
