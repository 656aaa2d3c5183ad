"""Host side of the big-tile weight-gradient kernel (``csrc/kernels/conv_wtile.hip``).

dW of a stride-1 3-D conv as an MFMA GEMM over output positions (K axis), one
workgroup per CU (4 MFMA waves + an LDS-DMA loader wave), double-buffered
tiles, XCD-aware column groups.  This module plans the tile (shape, k-steps,
LDS), builds the k-row order that keeps the transposed halo reads bank-conflict
free (every aligned group of 8 k-rows has 8 distinct halo positions mod 8) and
launches the kernel.

Reference parity: the weight gradient of Keras ``Conv3D`` (reference
``model/input.py:294``, TF autodiff); ``ops/conv.py`` keeps the conv_halo
wgrad as the fallback and A/B partner.
"""
from __future__ import annotations

import math
import os
import threading
from dataclasses import dataclass

import numpy as np
import torch

from .. import _native
from . import conv_tile

LDS_MAX = 160 * 1024
N_CUS = 256
_LOCK = threading.Lock()
_PLANS: dict = {}
_TABS: dict = {}
_SCHED: dict = {}
_ZERO: dict = {}


@dataclass(frozen=True)
class WPlan:
    TD: int
    TH: int
    TW: int
    HPpad: int
    kst: int
    nacc: int
    ntg: int
    G: int
    workers: int
    BUF: int
    cost: float
    nw: int = 4      # MFMA waves per workgroup: 4 (+ a loader wave) or 8 (no loader)
    c8: bool = False  # 8 input channels (the space-to-depth stem): two taps per B fragment
    ks2: bool = False  # k-steps split between the wave halves (twice the fragments per wave)
    sp: bool = False   # sub-pixel decoder form (ops/subpixel.py): wave = parity class, 2 slices

    @property
    def xr(self) -> int:
        """Halo bytes per position."""
        return 16 if self.c8 else 32

    @property
    def rows(self) -> int:
        return self.TD * self.TH * self.TW


def mode() -> str:
    """FN_WTILE: 1 (default) = deterministic per-shape choice vs conv_halo wgrad (ops/tuning.py),
    2 = always, 0 = off."""
    return os.environ.get("FN_WTILE", "1")


def _nacc(K: int, T: int, nw: int = 4) -> int | None:
    if nw == 8:                                   # 8 waves x nacc taps per workgroup
        if K not in (32, 64):
            return None
        for a in ((4, 8, 16) if K == 32 else (4, 8)):
            if T <= 8 * a:
                return a
        return 16 if K == 32 else 8
    if K == 16:
        return 16
    if K == 64:
        return 8
    if K == 32:
        def used(a):
            return T / (math.ceil(T / (4 * a)) * 4 * a)
        return 8 if used(8) >= 1.15 * used(16) else 16
    return None


def plan(spec) -> WPlan | None:
    if mode() == "0" or (spec.sd, spec.sh, spec.sw, spec.dd, spec.dh, spec.dw) != (1,) * 6:
        return None
    key = (spec.N, spec.D, spec.H, spec.W, spec.C, spec.K, spec.KD, spec.KH, spec.KW, spec.OD, spec.OH, spec.OW)
    if key in _PLANS:
        return _PLANS[key]
    p = _plan(spec)
    with _LOCK:
        _PLANS[key] = p
    return p


def ks2_enabled() -> bool:
    """FN_WTILE_KS2: 1 (default) = split the k-steps between the wave halves where a wave
    would otherwise hold 4 fragments (T <= 32 taps, or the 8-channel stem), 0 = off."""
    return os.environ.get("FN_WTILE_KS2", "1") != "0"


def nwaves() -> int:
    """FN_WTILE_NW: 8 (default) = the loaderless 8-MFMA-wave variant, 4 = 4 MFMA waves + loader."""
    return int(os.environ.get("FN_WTILE_NW", "8"))


def _plan(spec):
    K, C = spec.K, spec.C
    T = spec.KD * spec.KH * spec.KW
    nw = nwaves()
    c8 = C == 8 and nw == 8 and K in (32, 64)
    ks2 = False
    if c8:                                        # 8 waves x 4 fragments x 2 taps per workgroup
        nacc, tpf = 4, 2
    else:
        tpf = 1
        nacc = _nacc(K, T, nw)
        if nacc is None and nw == 8:
            nw, nacc = 4, _nacc(K, T)
        if nacc is None or C % 16:
            return None
    if T < 2:
        return None
    if nw == 8 and nacc == 4 and ks2_enabled() and (K == 32 or (K == 64 and not c8)) and T <= 4 * 8 * tpf:
        ks2, nacc = True, 8                       # 4 waves x 8 fragments per k-step stream
    ntg = -(-T // ((nw // 2 if ks2 else nw) * nacc * tpf))
    G = ntg * (1 if c8 else C // 16)
    xr, hq = (16, 64) if c8 else (32, 32)
    if 8 * G > 63:
        return None
    workers = max(1, N_CUS // (8 * G))
    OD, OH, OW = spec.OD, spec.OH, spec.OW
    MT = K // 16
    best = None
    tw_opts = sorted({OW} | {-(-OW // k) for k in range(2, 6) if -(-OW // k) >= 8})
    for TW in tw_opts:
        for TD in range(1, OD + 1):
            for TH in range(1, OH + 1):
                rows = TD * TH * TW
                if rows > 1024:
                    break
                kst = -(-rows // 32)
                if rows < 0.85 * kst * 32 or rows < 96:
                    continue
                HH, HW = TH + spec.KH - 1, TW + spec.KW - 1
                HP = (TD + spec.KD - 1) * HH * HW
                if max(TD + spec.KD - 1, HH, HW) > 255:
                    continue
                HPpad = -(-HP // hq) * hq
                BUF = -(-(HPpad * xr + kst * 32 * K * 2) // 1024) * 1024
                lds = 2 * BUF + 64 + kst * 32 * 12 + HPpad * 8        # + row / position / offset tables
                if lds > LDS_MAX:
                    continue
                tiles = spec.N * -(-OD // TD) * -(-OH // TH) * -(-OW // TW)
                jobs = math.ceil(math.ceil(tiles / 8) / workers)
                mfma = kst * nacc * MT * 16 * (2 if nw == 8 else 1) + 400   # per SIMD per job
                loader = 600 + (HPpad * xr // 1024 + kst * K // 16) * 60
                cost = jobs * max(mfma, loader) * (1.0 + 0.02 * HP / rows)   # halo re-reads (L2 traffic)
                if best is None or cost < best.cost:
                    best = WPlan(TD, TH, TW, HPpad, kst, nacc, ntg, G, workers, BUF, float(cost), nw, c8, ks2)
    return best


def tables(p: WPlan, kdims: tuple) -> tuple[np.ndarray, np.ndarray]:
    """(rowtab int32 [kst*32, 2], postab int32 [HPpad]).

    rowtab: per k-row (byte offset xr*hpos of its tap-0 halo position, packed tile coords
    td<<16 | th<<8 | tw, or -1 for a dummy row), ordered so every aligned group of 8 rows
    (one LDS cycle of a transposed read) touches 64 distinct banks: 32-B positions need 8
    distinct hpos mod 8; 16-B positions (c8) are read at hpos and hpos + 1 (the tap pair
    2i, 2i + 1 of a fragment, adjacent in kw), so a group takes 8 distinct residues mod 16
    of one parity.  Dummies take a missing residue (a real halo position).
    postab: packed halo coords hd<<16 | hh<<8 | hw per position, -1 past the halo."""
    key = (p, tuple(kdims))
    t = _TABS.get(key)
    if t is not None:
        return t
    KD, KH, KW = kdims
    HH, HW = p.TH + KH - 1, p.TW + KW - 1
    td, th, tw = np.meshgrid(np.arange(p.TD), np.arange(p.TH), np.arange(p.TW), indexing="ij")
    hpos = ((td * HH + th) * HW + tw).reshape(-1)
    pk = ((td << 16) | (th << 8) | tw).reshape(-1)
    ngroups = p.kst * 4
    groups = [[None] * 8 for _ in range(ngroups)]
    extra = []
    if p.c8:
        # group gi holds residues 2s + (gi & 1) (mod 16) in slot s
        buckets = [list(zip(hpos[hpos % 16 == r].tolist(), pk[hpos % 16 == r].tolist())) for r in range(16)]
        for r in range(16):
            par, s = r & 1, r >> 1
            for i, item in enumerate(buckets[r]):
                gi = 2 * i + par
                if gi < ngroups:
                    groups[gi][s] = item
                else:
                    extra.append(item)
        mod = 16
    else:
        buckets = [list(zip(hpos[hpos % 8 == r].tolist(), pk[hpos % 8 == r].tolist())) for r in range(8)]
        for r in range(8):
            for i, item in enumerate(buckets[r]):
                if i < ngroups:
                    groups[i][r] = item
                else:
                    extra.append(item)
        mod = 8
    for gr in groups:                             # overflow rows fill free slots (a conflict, not an error)
        for s in range(8):
            if gr[s] is None and extra:
                gr[s] = extra.pop()
    assert not extra, "row table overflow"
    for gi, gr in enumerate(groups):
        for s in range(8):
            if gr[s] is None:
                used = {x[0] % mod for x in gr if x is not None}
                want = 2 * s + (gi & 1) if p.c8 else s
                cand = [want] if want not in used else [r for r in range(mod) if r not in used]
                gr[s] = ((cand[0] if cand else 0), -1)
    rows = np.asarray([(h * p.xr, k) for gr in groups for (h, k) in gr], dtype=np.int32)
    HP = (p.TD + KD - 1) * HH * HW
    pos = np.full(p.HPpad, -1, dtype=np.int32)
    q = np.arange(HP)
    pos[:HP] = ((q // (HH * HW)) << 16) | (((q // HW) % HH) << 8) | (q % HW)
    with _LOCK:
        _TABS[key] = (rows, pos)
    return rows, pos


def _dev(cache: dict, key, make):
    t = cache.get(key)
    if t is None:
        t = make()
        with _LOCK:
            cache[key] = t
    return t


_PART: dict = {}
_RETIRED: list = []


def _partials(dev, stream: int, n: int) -> torch.Tensor:
    """fp32 scratch for the per-(XCD, worker) partial weight gradients (one buffer per device
    and stream, grown to the largest layer; the kernel overwrites what it reads)."""
    key = (str(dev), stream)
    t = _PART.get(key)
    if t is None or t.numel() < n:
        t = torch.empty(n, dtype=torch.float32, device=dev)
        with _LOCK:
            if key in _PART:                     # a captured hipGraph may still name the old one
                _RETIRED.append(_PART[key])
            _PART[key] = t
    return t


def plan_subpixel(N: int, cells: tuple, C: int, K: int) -> WPlan | None:
    """Tile plan of the sub-pixel decoder weight gradient: rows = low-res cells (all 8 parity
    classes of a cell in one 512-B dy row), x halo = two 16-channel planes of the 3^3
    footprint (pad 1), 16 fragments per wave (8 folded taps x 2 slices)."""
    if K != 32 or C % 32 or nwaves() != 8:
        return None
    key = ("sp", N, tuple(cells), C, K)
    if key in _PLANS:
        return _PLANS[key]
    OD, OH, OW = cells
    G = C // 32
    workers = max(1, N_CUS // (8 * G))
    best = None
    for TW in sorted({OW} | {-(-OW // k) for k in range(2, 6) if -(-OW // k) >= 8}):
        for TD in range(1, OD + 1):
            for TH in range(1, OH + 1):
                rows = TD * TH * TW
                if rows > 1024:
                    break
                kst = -(-rows // 32)
                if rows < 0.85 * kst * 32 or rows < 64:
                    continue
                HP = (TD + 2) * (TH + 2) * (TW + 2)
                HPpad = -(-HP // 32) * 32
                BUF = -(-(2 * HPpad * 32 + kst * 32 * 8 * K * 2) // 1024) * 1024
                lds = 2 * BUF + 64 + kst * 32 * 12 + HPpad * 8
                if lds > LDS_MAX:
                    continue
                tiles = N * -(-OD // TD) * -(-OH // TH) * -(-OW // TW)
                jobs = math.ceil(math.ceil(tiles / 8) / workers)
                mfma = kst * 16 * 2 * 16 * 2 + 400                  # per SIMD per job (2 waves)
                dma = 600 + (2 * HPpad * 32 + kst * 32 * 8 * K * 2) // 1024 * 45
                cost = jobs * max(mfma, dma) * (1.0 + 0.02 * HP / rows)
                if best is None or cost < best.cost:
                    best = WPlan(TD, TH, TW, HPpad, kst, 16, 1, G, workers, BUF, float(cost), 8, sp=True)
    with _LOCK:
        _PLANS[key] = best
    return best


def conv_wgrad_subpixel(dsh: torch.Tensor, x5: torch.Tensor, p: WPlan) -> torch.Tensor:
    """Per-class folded weight gradients [8, K, 2, 2, 2, C] (fp32) of the sub-pixel decoder:
    ``dsh`` = the shifted space-to-depth dy [N, D+1, H+1, W+1, 8K], ``x5`` = the low-res input
    [N, D, H, W, C] (ops/subpixel.py; :func:`subpixel.fold_weight_grad` gives dW)."""
    assert p.sp
    N, D, H, W, C = x5.shape
    K = dsh.shape[-1] // 8
    assert dsh.shape == (N, D + 1, H + 1, W + 1, 8 * K) and dsh.is_contiguous() and x5.is_contiguous()
    kd = (3, 3, 3)
    dev = x5.device
    rt_np, pt_np = tables(p, kd)
    rt = _dev(_TABS, ("rt", p, kd, str(dev)), lambda: torch.from_numpy(rt_np).to(dev))
    pt = _dev(_TABS, ("pt", p, kd, str(dev)), lambda: torch.from_numpy(pt_np).to(dev))
    zp = _dev(_ZERO, str(dev), lambda: torch.zeros(64, dtype=torch.bfloat16, device=dev))
    st = _native.stream(x5)
    sched = conv_tile.counters(_SCHED, _LOCK, dev, st, 64)
    dw = torch.zeros(8 * K, 8, C, dtype=torch.float32, device=dev)
    part = _partials(dev, st, 8 * p.workers * dw.numel())
    geom = [N, D, H, W, C, D, H, W, K, 3, 3, 3, 1, 1, 1, p.TD, p.TH, p.TW, p.HPpad, p.kst, 2 * p.HPpad * 32, p.BUF,
            p.G, p.ntg]
    _native.kernels().conv_wtile(x5.data_ptr(), dsh.data_ptr(), dw.data_ptr(), part.data_ptr(), rt.data_ptr(),
                                 pt.data_ptr(), zp.data_ptr(), geom, flags(p), p.workers, sched.data_ptr(), st,
                                 [x5.numel(), dsh.numel(), dw.numel(), rt.numel() // 2, pt.numel(), part.numel()])
    return dw.reshape(8, K, 2, 2, 2, C)


def geometry(p: WPlan, spec) -> list[int]:
    XB = p.HPpad * p.xr
    return [spec.N, spec.D, spec.H, spec.W, spec.C, spec.OD, spec.OH, spec.OW, spec.K, spec.KD, spec.KH, spec.KW,
            spec.pd, spec.ph, spec.pw, p.TD, p.TH, p.TW, p.HPpad, p.kst, XB, p.BUF, p.G, p.ntg]


def flags(p: WPlan) -> int:
    """The launcher's variant word: nacc | 8 << 8 (8 waves) | 1 << 12 (8-channel form)
    | 1 << 13 (k-steps split between the wave halves)."""
    return (p.nacc | (p.nw << 8 if p.nw == 8 else 0) | (1 << 12 if p.c8 else 0) | (1 << 13 if p.ks2 else 0)
            | (1 << 14 if p.sp else 0))


def prologue_ok(p: WPlan) -> bool:
    """The plan's kernel form can normalise its x halos itself (BN prologue: 16-channel slices --
    not the 8-channel space-to-depth stem form nor the sub-pixel form; experiment builds only)."""
    return not p.c8 and not p.sp and bool(_native.kernels().conv_wtile_prologue_built())


def conv_wgrad(dy5: torch.Tensor, x5: torch.Tensor, spec, p: WPlan, out=None, wdot=None, pro=None):
    """dW fp32 [K, KD, KH, KW, C] on the big-tile wgrad kernel (accumulated into ``out``
    when given: a zeroed contiguous fp32 tensor of that size, e.g. the flat gradient).
    ``wdot`` (the layer's fp32 weights, that layout): returns ``(dW, S partials)`` where the
    partial slab [blocks, C] of S = sum W . dW comes from the kernel's reduce pass (the BN
    statistics identity, ``bn_pool.hip``; no separate bn_wdot launch).
    ``pro`` = (prm [4, C], act): ``x5`` is a BN's pre-normalisation y and the conv's input is
    act(y * prm[2] + prm[3]), applied by the kernel to every landed x halo (:func:`prologue_ok`)."""
    kd = (spec.KD, spec.KH, spec.KW)
    dev = x5.device
    rt_np, pt_np = tables(p, kd)
    rt = _dev(_TABS, ("rt", p, kd, str(dev)), lambda: torch.from_numpy(rt_np).to(dev))
    pt = _dev(_TABS, ("pt", p, kd, str(dev)), lambda: torch.from_numpy(pt_np).to(dev))
    zp = _dev(_ZERO, str(dev), lambda: torch.zeros(64, dtype=torch.bfloat16, device=dev))
    st = _native.stream(x5)
    sched = conv_tile.counters(_SCHED, _LOCK, dev, st, 64)
    dw = out if out is not None else torch.zeros(spec.K, spec.taps, spec.C, dtype=torch.float32, device=dev)
    part = _partials(dev, st, 8 * p.workers * (2 if p.ks2 else 1) * dw.numel())
    wsrc = wdp = None
    if wdot is not None and 256 % spec.C == 0:
        wsrc = wdot.detach().float().contiguous()
        wdp = torch.empty(-(-dw.numel() // 256), spec.C, dtype=torch.float32, device=dev)
    ext = [x5.numel(), dy5.numel(), dw.numel(), rt.numel() // 2, pt.numel(), part.numel()]
    ext += [wsrc.numel(), wdp.numel()] if wsrc is not None else [0, 0]
    pk = {}
    if pro is not None:
        prm, pact = pro
        assert prologue_ok(p) and prm.is_contiguous() and prm.shape == (4, spec.C) and prm.dtype == torch.float32
        ext.append(2 * spec.C)
        pk = dict(pst=prm[2].data_ptr(), pact=int(pact))
    _native.kernels().conv_wtile(x5.data_ptr(), dy5.data_ptr(), dw.data_ptr(), part.data_ptr(), rt.data_ptr(),
                                 pt.data_ptr(), zp.data_ptr(), geometry(p, spec), flags(p), p.workers, sched.data_ptr(),
                                 st, ext, _native.ptr(wsrc), _native.ptr(wdp), **pk)
    dw = dw.reshape(spec.K, spec.KD, spec.KH, spec.KW, spec.C)
    return dw if wdot is None else (dw, wdp)


def choose(spec, run_wtile, run_halo) -> bool:
    """True when this kernel should run the weight gradient of ``spec``: FN_WTILE=2 always,
    otherwise the deterministic per-shape selection of :mod:`.tuning`."""
    if mode() == "2":
        return True
    from . import tuning

    return tuning.select("wgrad", spec, run_wtile, run_halo)
