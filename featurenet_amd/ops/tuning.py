"""Deterministic per-shape kernel selection for gfx950: a rule plus measured exceptions.

Several convolution shapes have two native implementations -- the big-tile kernels
(``conv_tile.hip`` forward / dgrad, ``conv_wtile.hip`` weight gradient) and the
older halo kernels (``conv_halo.hip``).  Round 2 picked between them by timing
each new shape once in-process, so two runs, two boxes or two data-parallel ranks
could run different kernels (different bf16 rounding, run-to-run variance).

Selection is now a pure function of the shape:

1. :data:`EXCEPTIONS` -- measured choices for shapes where the rule is wrong
   (``scripts/bench_conv_layers.py`` on 1x MI355X, batch 128; each entry cites the
   profile that decided it).  It is empty: on every FeatureNet-3D and search-space
   shape measured in rounds 2-4 the big-tile kernels beat the halo kernels
   (``profiles/r4_m32_ab.md`` has the round-4 layer times of both);
2. the rule: the big-tile kernel whenever it can plan the shape.

``FN_KERNEL_SELECT=autotune`` restores per-shape timing for shapes without an exception
(research / new shapes); under data parallelism :func:`sync_from_rank0` then makes
every rank adopt rank 0's decisions before the step is captured.  Every decision is
logged once per shape (``kernel_choice`` events, :mod:`featurenet_amd.utils.events`).

Reference parity: kernel choice never changes the math -- the same Keras
``Conv2D``/``Conv3D`` (reference ``model/input.py:294``) either way.
"""
from __future__ import annotations

import os
import threading

import torch

_LOCK = threading.Lock()
_DECIDED: dict = {}      # (kind, shape key) -> bool, every decision taken in this process
_LOGGED: set = set()

# (kind, D, H, W, C, K, KD, KH, KW, sd, sh, sw, pd, ph, pw) -> True (big-tile kernel) / False (halo)
# Only exceptions to the rule "big-tile whenever it plans" are listed (none measured so far).
EXCEPTIONS: dict = {
}


def shape_key(spec) -> tuple:
    """The spec without the batch: kernel choice is per layer shape, not per batch size."""
    return (spec.D, spec.H, spec.W, spec.C, spec.K, spec.KD, spec.KH, spec.KW, spec.sd, spec.sh, spec.sw,
            spec.pd, spec.ph, spec.pw)


def mode() -> str:
    return os.environ.get("FN_KERNEL_SELECT", "table")


def _log(kind: str, spec, choice: bool, source: str) -> None:
    key = (kind, shape_key(spec))
    if key in _LOGGED:
        return
    _LOGGED.add(key)
    try:
        from ..utils.events import default_log

        default_log().emit("kernel_choice", kind=kind, shape=list(shape_key(spec)), batch=spec.N,
                           kernel="tile" if choice else "halo", source=source)
    except Exception:  # noqa: BLE001 - logging must never break a forward pass
        pass


def _time_ms(fn, reps: int = 3) -> float:
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


def select(kind: str, spec, run_tile=None, run_other=None) -> bool:
    """True when the big-tile kernel should run ``kind`` ('fwd' | 'dgrad' | 'wgrad') of ``spec``."""
    key = (kind, shape_key(spec))
    c = _DECIDED.get(key)
    if c is not None:
        return c
    src = "table"
    tk = (kind,) + key[1]
    if tk in EXCEPTIONS:
        c = bool(EXCEPTIONS[tk])
    elif mode() == "autotune" and run_tile is not None and run_other is not None and \
            not torch.cuda.is_current_stream_capturing():
        c = _time_ms(run_tile) <= _time_ms(run_other)
        src = "autotune"
    else:
        c, src = True, "rule"
    with _LOCK:
        _DECIDED[key] = c
    _log(kind, spec, c, src)
    return c


def predict(kind: str, spec):
    """What :func:`select` will return for ``kind`` of ``spec`` without timing anything: True /
    False, or None when only an autotune measurement can tell."""
    key = (kind, shape_key(spec))
    c = _DECIDED.get(key)
    if c is not None:
        return c
    tk = (kind,) + key[1]
    if tk in EXCEPTIONS:
        return bool(EXCEPTIONS[tk])
    return None if mode() == "autotune" else True


def decisions() -> dict:
    return dict(_DECIDED)


def sync_from_rank0(group=None) -> int:
    """Data parallel: every rank adopts rank 0's kernel decisions (call after the eager warmup
    steps, before capturing the step).  Returns the number of decisions received."""
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return 0
    obj = [sorted(_DECIDED.items())] if dist.get_rank(group) == 0 else [None]
    dist.broadcast_object_list(obj, src=0, group=group)
    with _LOCK:
        _DECIDED.clear()
        _DECIDED.update(dict(obj[0]))
    return len(obj[0])
