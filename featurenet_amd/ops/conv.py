"""Convolution op: native implicit-GEMM HIP kernels on GPU, reference on CPU.

Reference parity: this op is what the reference builds with Keras
``Conv1D/Conv2D`` (``model/input.py:294-306``) and the 1x1 channel projection
inside ``Combination`` (``model/operation.py:179-186``); the north-star
Conv3d layers of FeatureNet-3D use the same code path.

GPU path:
  forward -> ``conv_halo`` (``csrc/kernels/conv_halo.hip``) for stride-1 convs
             with >= 8 taps and C % 16 == 0 (LDS-staged input halo tiles),
             else ``igemm_fwd`` (``conv_igemm.hip``, gathered im2col);
             both fuse bias+activation or emit BN statistics
  dgrad   -> ``conv_halo`` on dy with the flipped, transposed kernel (stride 1)
             or ``igemm_fwd`` in transposed-conv mode (negated tap table)
  wgrad   -> ``conv_halo_wgrad`` (stride 1, Cout <= 64: halo tiles, persistent
             workgroups, per-workgroup partials summed in a fixed order) or ``igemm_wgrad``
             (split-m partials, summed in a fixed order)
``FEATURENET_CONV_HALO=0`` disables the halo path (A/B checks).
"""
from __future__ import annotations

import dataclasses
import math
import os
import threading

import numpy as np
import torch
import torch.nn.functional as F

from .. import _native
from . import bnfuse
from . import conv_tile
from . import conv_wtile
from . import packs
from . import reference as ref
from ..training.flat import grad_target
from .spec import ConvSpec, act_code

_TAB_LOCK = threading.Lock()
# the space-to-depth forward pads K (FeatureNet-3D stem: 512 vs 343); it is taken when
# the padded K is at most this multiple of the real one (else the packed-W gather runs)
S2D_FWD_RATIO = 1.5
_TAB_CACHE: dict = {}


# ---------------------------------------------------------------------------
# tap tables
# ---------------------------------------------------------------------------
def _fwd_table(spec: ConvSpec, vec: bool) -> np.ndarray:
    C = spec.C
    kd, kh, kw, ci = np.meshgrid(np.arange(spec.KD), np.arange(spec.KH), np.arange(spec.KW), np.arange(C),
                                 indexing="ij")
    kd, kh, kw, ci = (a.reshape(-1) for a in (kd, kh, kw, ci))
    zd, zh, zw = kd * spec.dd, kh * spec.dh, kw * spec.dw
    off = ((zd * spec.H + zh) * spec.W + zw) * C + ci
    tab = np.stack([off, zd, zh, zw], axis=1).astype(np.int64)
    if vec:
        tab = tab[::8]
    return tab


GM_SCALAR, GM_VEC, GM_PACKW = 0, 1, 2


def gather_mode(spec: ConvSpec) -> int:
    """Kernel gather mode for the forward / wgrad im2col of ``x``."""
    if spec.C % 8 == 0:
        return GM_VEC
    if spec.C < 8 and spec.dw == 1:
        return GM_PACKW
    return GM_SCALAR


def packw_row(spec: ConvSpec) -> int:
    """Elements per (kd, kh) row of the packed-W K layout (KW*C rounded up to 8)."""
    return (spec.KW * spec.C + 7) // 8 * 8


def _packw_table(spec: ConvSpec) -> np.ndarray:
    C, R = spec.C, packw_row(spec)
    rows = []
    for kd in range(spec.KD):
        for kh in range(spec.KH):
            zd, zh = kd * spec.dd, kh * spec.dh
            base = ((zd * spec.H + zh) * spec.W) * C
            for p0 in range(0, R, 8):
                lo = p0 // C
                hi = (p0 + 7) // C
                rows.append((base + p0, (zd << 16) | zh, (lo << 16) | hi, p0))
    return np.asarray(rows, dtype=np.int64)


def kdim_gather(spec: ConvSpec) -> int:
    return spec.KD * spec.KH * packw_row(spec) if gather_mode(spec) == GM_PACKW else spec.kdim


def _ig_pack_geom(spec: ConvSpec, mode: int) -> tuple[int, int, int]:
    """(rows, ld, R) of the igemm_pack_w layout ``mode``."""
    if mode == 2:
        R = packw_row(spec)
        return spec.K, spec.KD * spec.KH * R, R
    return (spec.C if mode == 1 else spec.K), ((spec.taps * (spec.K if mode == 1 else spec.C)) + 7) // 8 * 8, 0


def _native_pack(w: torch.Tensor, spec: ConvSpec, mode: int) -> tuple[torch.Tensor, int]:
    """One igemm_pack_w launch: fp32 ``w`` [K0, KD, KH, KW, C0] (K0 <= spec.K, C0 <= spec.C: the
    missing rows / channels are zeros) -> the bf16 B rows of mode 0 (forward), 1 (dgrad:
    [C][taps*K]) or 2 (packed-W forward), row stride padded to 8.  Inside a :class:`pack_scope`
    the model's forward has made it already (one launch for every layer)."""
    hit = _pack_lookup(w, spec, mode)
    if hit is not None:
        return hit
    wf = w.detach().float().contiguous()
    rows, ld, R = _ig_pack_geom(spec, mode)
    out = torch.empty(rows, ld, dtype=torch.bfloat16, device=w.device)
    _native.kernels().igemm_pack_w(wf.data_ptr(), out.data_ptr(), wf.shape[0], wf.shape[-1], spec.K, spec.taps, spec.C,
                                   mode, ld, spec.KW, R, _native.stream(wf), [wf.numel(), out.numel()])
    _pack_record(w, spec, mode)
    return out, ld


# one-launch packing of a model forward's weights (ops/packs.py): the gather / halo layouts
# (kinds 0-2: igemm_pack_w modes, 3 / 4: halo forward / dgrad)
_pack_lookup = packs.lookup
_pack_record = packs.record
pack_scope = packs.pack_scope
_PK_GENS, _PK_TLS = packs.GENS, packs.TLS


def _pack_job(p: torch.Tensor, spec: ConvSpec, kind: int):
    """(job row, output, cache value) of one recorded gather / halo pack."""
    K0, C0 = p.shape[0], p.shape[-1]
    T = spec.taps
    if kind <= 2:
        rows, ld, R = _ig_pack_geom(spec, kind)
        out = torch.empty(rows, ld, dtype=torch.bfloat16, device=p.device)
        a = [K0, C0, spec.K, T, spec.C, ld, spec.KW, R, 0]
        val = (out, ld)
    else:
        dgrad = kind == 4
        ncol, csrc = (spec.C, spec.K) if dgrad else (spec.K, spec.C)
        cs = halo_cs(csrc)
        tps = 128 // cs
        Tp = (T + tps - 1) // tps * tps
        out = torch.empty(ncol, csrc * Tp, dtype=torch.bfloat16, device=p.device)
        a = [K0, C0, spec.K, T, spec.C, cs, Tp, 0, 0]
        val = out
    return [p.data_ptr(), out.data_ptr(), kind] + a, out, val


packs.register((0, 1, 2, 3, 4), lambda p, spec, kind: _pack_job(p, spec, kind), lambda spec, kind: kind in (1, 4))


def pad_to_spec(w: torch.Tensor, spec: ConvSpec) -> torch.Tensor:
    """``w`` zero-padded to ``spec``'s output / input channel counts (no copy when they match)."""
    return pad_weight(w, cin=spec.C, cout=spec.K)


def pack_weight_rows(w: torch.Tensor, spec: ConvSpec) -> tuple[torch.Tensor, int]:
    """Forward B operand [Cout, Kdim'] in the gather layout of ``spec`` (``w`` may have fewer
    output / input channels than ``spec``: zero rows / channels)."""
    if w.is_cuda and _native.kernels_available():
        return _native_pack(w, spec, 2 if gather_mode(spec) == GM_PACKW else 0)
    w = pad_to_spec(w, spec)
    if gather_mode(spec) == GM_PACKW:
        R = packw_row(spec)
        out = torch.zeros(spec.K, spec.KD * spec.KH, R, dtype=torch.bfloat16, device=w.device)
        out[:, :, : spec.KW * spec.C] = w.reshape(spec.K, spec.KD * spec.KH, spec.KW * spec.C)
        return out.reshape(spec.K, -1), spec.KD * spec.KH * R
    return _pack_rows(w.reshape(spec.K, spec.kdim))


def _dgrad_table(spec: ConvSpec, vec: bool) -> np.ndarray:
    """k' = tap*K + co over dy (dims OD', OH', OW' = zero-inserted dy)."""
    K = spec.K
    ODu, OHu, OWu = _dgrad_src_dims(spec)
    kd, kh, kw, co = np.meshgrid(np.arange(spec.KD), np.arange(spec.KH), np.arange(spec.KW), np.arange(K),
                                 indexing="ij")
    kd, kh, kw, co = (a.reshape(-1) for a in (kd, kh, kw, co))
    zd, zh, zw = -kd * spec.dd, -kh * spec.dh, -kw * spec.dw
    off = ((zd * OHu + zh) * OWu + zw) * K + co
    tab = np.stack([off, zd, zh, zw], axis=1).astype(np.int64)
    if vec:
        tab = tab[::8]
    return tab


def _dgrad_src_dims(spec: ConvSpec) -> tuple[int, int, int]:
    return ((spec.OD - 1) * spec.sd + 1, (spec.OH - 1) * spec.sh + 1, (spec.OW - 1) * spec.sw + 1)


def _table(spec: ConvSpec, kind: str, vec: bool, device) -> torch.Tensor:
    key = (spec, kind, vec, str(device))
    t = _TAB_CACHE.get(key)
    if t is None:
        if kind == "fwd":
            arr = _packw_table(spec) if vec == GM_PACKW else _fwd_table(spec, vec == GM_VEC)
        else:
            arr = _dgrad_table(spec, vec)
        if np.abs(arr).max(initial=0) >= 2**31:
            raise ValueError("conv tap offsets overflow int32")
        t = torch.from_numpy(arr.astype(np.int32)).to(device)
        with _TAB_LOCK:
            _TAB_CACHE[key] = t
    return t


def _geom_fwd(spec: ConvSpec) -> list[int]:
    return [spec.OD, spec.OH, spec.OW, spec.sd, spec.sh, spec.sw, -spec.pd, -spec.ph, -spec.pw,
            spec.D, spec.H, spec.W, spec.C, spec.KW * spec.C]


def _geom_dgrad(spec: ConvSpec) -> list[int]:
    ODu, OHu, OWu = _dgrad_src_dims(spec)
    return [spec.D, spec.H, spec.W, 1, 1, 1, spec.pd, spec.ph, spec.pw, ODu, OHu, OWu, spec.K, 0]


def _pack_rows(mat: torch.Tensor) -> tuple[torch.Tensor, int]:
    """bf16 [R, K] with the row stride padded to a multiple of 8 (zero tail)."""
    R, K = mat.shape
    ld = (K + 7) // 8 * 8
    if ld == K:
        return mat.to(torch.bfloat16).contiguous(), ld
    out = torch.zeros(R, ld, dtype=torch.bfloat16, device=mat.device)
    out[:, :K] = mat
    return out, ld


# ---------------------------------------------------------------------------
# LDS-halo path (stride-1 convs)
# ---------------------------------------------------------------------------
LDS_BUDGET = 80 * 1024      # two workgroups per CU (160 KiB LDS)
_PLAN_CACHE: dict = {}


def halo_cs(C: int) -> int:
    """Channels per LDS halo slice of the halo kernels: 16, 8 (8-channel inputs) or 0 (unsupported)."""
    return 16 if C % 16 == 0 else (8 if C % 8 == 0 else 0)


def _fwd_halo_budget(ncol: int, cs: int = 16) -> int:
    bn = 32 if ncol <= 32 else 64
    # halo + 4 B/position decode table, expressed in 32-B (16-channel bf16) positions
    return int((LDS_BUDGET - 2 * bn * 128 * 2 - 1024) * 32 / (cs * 2 + 4))


def _wgrad_halo_budget(cout: int, cs: int = 16) -> int:
    mt = (cout + 15) // 16
    return int((LDS_BUDGET - 256 * (16 * mt + 16) * 2 - 2048 - 64) * 32 / (cs * 2 + 4))


def _plan_tw(OD, OH, OW, KD, KH, KW, max_bytes, TW):
    best, best_score = None, -1.0
    if TW > 256:
        return best, best_score
    for TD in range(1, OD + 1):
        for TH in range(1, OH + 1):
            rows = TD * TH * TW
            if rows > 256:
                break
            halo = (TD + KD - 1) * (TH + KH - 1) * (TW + KW - 1) * 32
            if halo > max_bytes:
                continue
            tiles = math.ceil(OD / TD) * math.ceil(OH / TH) * math.ceil(OW / TW)
            score = OD * OH * OW / (tiles * 256.0) - 1e-9 * halo
            if score > best_score:
                best, best_score = (TD, TH, TW), score
    return best, best_score


def halo_plan(OD: int, OH: int, OW: int, KD: int, KH: int, KW: int, max_bytes: int = 56 * 1024,
              wsplit: bool = True):
    """Output tile (TD, TH, TW) maximising MFMA row utilisation (rows = TD*TH*TW <= 256)
    with the halo (counted at 32 B = 16 bf16 channels per position) <= max_bytes; None
    when no tile fits.  Tiles span the full output width (TW = OW) unless that leaves
    the 256-row MFMA tile under 75 % used (wide outputs: 128^3 inference, where a
    5^3 halo of full 57-wide rows only fits a 57-row tile), in which case OW is split
    into equal column tiles."""
    key = (OD, OH, OW, KD, KH, KW, max_bytes, wsplit)
    if key in _PLAN_CACHE:
        return _PLAN_CACHE[key]
    best, best_score = _plan_tw(OD, OH, OW, KD, KH, KW, max_bytes, OW)
    if wsplit and best_score < 0.75:
        for k in range(2, 9):
            TW = -(-OW // k)
            if TW < 8:
                break
            cand, score = _plan_tw(OD, OH, OW, KD, KH, KW, max_bytes, TW)
            if score > best_score + 0.02:          # a split must pay for its extra halo columns
                best, best_score = cand, score
    _PLAN_CACHE[key] = best
    return best


def _halo_enabled() -> bool:
    return os.environ.get("FEATURENET_CONV_HALO", "1") != "0"


def halo_fwd_plan(spec: ConvSpec):
    if not _halo_enabled() or (spec.sd, spec.sh, spec.sw, spec.dd, spec.dh, spec.dw) != (1,) * 6:
        return None
    if not halo_cs(spec.C) or spec.K < 16 or spec.taps < 8:
        return None
    return halo_plan(spec.OD, spec.OH, spec.OW, spec.KD, spec.KH, spec.KW, _fwd_halo_budget(spec.K, halo_cs(spec.C)))


def halo_dgrad_plan(spec: ConvSpec):
    if not _halo_enabled() or (spec.sd, spec.sh, spec.sw, spec.dd, spec.dh, spec.dw) != (1,) * 6:
        return None
    if spec.K % 16 or spec.C < 16 or spec.taps < 8:
        return None
    return halo_plan(spec.D, spec.H, spec.W, spec.KD, spec.KH, spec.KW, _fwd_halo_budget(spec.C, 16))


def halo_pack(w: torch.Tensor, spec: ConvSpec, dgrad: bool) -> torch.Tensor:
    """Halo-kernel B operand of a conv weight [K0, KD, KH, KW, C0] (K0 <= spec.K, C0 <= spec.C:
    missing output / input channels are zeros): forward layout, or the dgrad layout (taps
    reversed, K <-> C); one HIP launch on GPU (or from the :class:`pack_scope` cache)."""
    if w.is_cuda and _native.kernels_available():
        kind = 4 if dgrad else 3
        hit = _pack_lookup(w, spec, kind)
        if hit is not None:
            return hit
        wf = w.detach().float().contiguous()
        ncol, csrc = (spec.C, spec.K) if dgrad else (spec.K, spec.C)
        cs = halo_cs(csrc)
        tps = 128 // cs
        Tp = (spec.taps + tps - 1) // tps * tps
        out = torch.empty(ncol, csrc * Tp, dtype=torch.bfloat16, device=w.device)
        _native.kernels().halo_pack_w(wf.data_ptr(), out.data_ptr(), wf.shape[0], wf.shape[-1], spec.K, spec.taps, spec.C,
                                      int(dgrad), 128, _native.stream(wf), [wf.numel(), out.numel()])
        _pack_record(w, spec, kind)
        return out
    w = pad_to_spec(w, spec)
    w3 = w.reshape(spec.K, spec.taps, spec.C)
    return halo_weights(w3.flip(1).permute(2, 1, 0) if dgrad else w3)


def halo_weights(w3: torch.Tensor) -> torch.Tensor:
    """[Ncol, T, Csrc] -> bf16 [Ncol, Csrc/CS * Tp * CS] in the halo kernel's k order
    (CS-channel slice, taps padded to a multiple of 128/CS, CS channels; CS = halo_cs(Csrc))."""
    n, T, c = w3.shape
    cs = halo_cs(c)
    tps = 128 // cs
    Tp = (T + tps - 1) // tps * tps
    out = torch.zeros(n, c // cs, Tp, cs, dtype=torch.bfloat16, device=w3.device)
    out[:, :, :T] = w3.reshape(n, T, c // cs, cs).permute(0, 2, 1, 3)
    return out.reshape(n, -1)


_TOFF_CACHE: dict = {}


def halo_tap_offsets(geom: list, device) -> torch.Tensor:
    """int32 [T8]: halo-position offset of every tap for a (kernel, tile) geometry."""
    key = (tuple(geom[5:]), str(device))
    t = _TOFF_CACHE.get(key)
    if t is None:
        OW, KD, KH, KW, TD, TH = geom[7], geom[8], geom[9], geom[10], geom[14], geom[15]
        TW = geom[16] if len(geom) > 16 else OW
        HH, HW = TH + KH - 1, TW + KW - 1
        T = KD * KH * KW
        offs = np.zeros((T + 15) // 16 * 16, dtype=np.int32)      # >= Tp for both slice widths
        kd, kh, kw = np.meshgrid(np.arange(KD), np.arange(KH), np.arange(KW), indexing="ij")
        offs[:T] = ((kd * HH + kh) * HW + kw).reshape(-1)
        t = torch.from_numpy(offs).to(device)
        with _TAB_LOCK:
            _TOFF_CACHE[key] = t
    return t


def halo_wgrad_plan(spec: ConvSpec):
    if not _halo_enabled() or (spec.sd, spec.sh, spec.sw, spec.dd, spec.dh, spec.dw) != (1,) * 6:
        return None
    if not halo_cs(spec.C) or spec.K % 8 or spec.K > 64 or spec.taps < 8:
        return None
    return halo_plan(spec.OD, spec.OH, spec.OW, spec.KD, spec.KH, spec.KW, _wgrad_halo_budget(spec.K, halo_cs(spec.C)))


_SCHED: dict = {}


def part_scratch(n: int, device) -> torch.Tensor:
    """fp32 scratch for the per-workgroup partial weight gradients of the wgrad kernels (every
    element is written by the kernel, then the rows are added into dW in a fixed order by
    ``fn_part_reduce``: bitwise-repeatable gradients, no float atomics)."""
    return torch.empty(max(1, int(n)), dtype=torch.float32, device=device)


def halo_sched(device, stream: int) -> torch.Tensor:
    """int32[64] tile-schedule counters of the halo kernel (one buffer per device and stream:
    kernels on one stream run in order, and every launch leaves the counters zero)."""
    return conv_tile.counters(_SCHED, _TAB_LOCK, device, stream, 64)


def halo_conv_wgrad(dy5, x5, spec: ConvSpec, plan, target_wgs: int = 512, out=None) -> torch.Tensor:
    """dW via LDS halo tiles; fp32 [K, KD, KH, KW, C] (accumulated into ``out`` when given:
    a zeroed contiguous fp32 tensor of that size, e.g. the parameter's flat gradient)."""
    TD, TH, TW = plan
    geom = [spec.N, spec.D, spec.H, spec.W, spec.C, spec.OD, spec.OH, spec.OW, spec.KD, spec.KH, spec.KW,
            spec.pd, spec.ph, spec.pw, TD, TH, TW]
    cs = halo_cs(spec.C)
    K = _native.kernels()
    per_tile = int(K.conv_halo_wgrad_yblocks(geom, spec.K)) * (spec.C // cs)
    dw = out if out is not None else torch.zeros(spec.K, spec.taps, spec.C, dtype=torch.float32, device=x5.device)
    st = _native.stream(x5)
    gx = max(1, target_wgs // per_tile)
    # per-workgroup partial weight gradients, added into dw in a fixed order (repeatable bits)
    part = part_scratch(int(K.conv_halo_wgrad_gx(geom, gx)) * spec.K * spec.taps * spec.C, x5.device)
    K.conv_halo_wgrad(dy5.data_ptr(), x5.data_ptr(), dw.data_ptr(), part.data_ptr(), geom, spec.K, gx, st,
                      [dy5.numel(), x5.numel(), dw.numel(), part.numel()])
    return dw.reshape(spec.K, spec.KD, spec.KH, spec.KW, spec.C)


def _halo_call(src5, wmat, bias, out, stats, geom, ncol, act):
    K = _native.kernels()
    if act and bias is None:
        bias = torch.zeros(ncol, dtype=torch.float32, device=src5.device)
    toffs = halo_tap_offsets(geom, src5.device)
    st = _native.stream(src5)
    K.conv_halo(src5.data_ptr(), wmat.data_ptr(), _native.ptr(bias), out.data_ptr(), _native.ptr(stats),
                toffs.data_ptr(), geom, ncol, act, halo_sched(src5.device, st).data_ptr(), st,
                [src5.numel(), wmat.numel(), out.numel(), toffs.numel()])


def halo_conv_fwd(x5, w, bias, spec: ConvSpec, act: int, want_stats: bool, plan):
    TD, TH, TW = plan
    geom = [spec.N, spec.D, spec.H, spec.W, spec.C, spec.OD, spec.OH, spec.OW, spec.KD, spec.KH, spec.KW,
            spec.pd, spec.ph, spec.pw, TD, TH, TW]
    wmat = halo_pack(w, spec, dgrad=False)
    y = torch.empty(spec.out_shape5, dtype=torch.bfloat16, device=x5.device)
    stats = None
    if want_stats:   # one (sum, sumsq) row per persistent workgroup
        stats = torch.empty(_native.kernels().conv_halo_workers(geom, spec.K), 2, spec.K, dtype=torch.float32,
                            device=x5.device)
    _halo_call(x5, wmat, bias, y, stats, geom, spec.K, act)
    return y, stats


def halo_conv_dgrad(dy5, w, spec: ConvSpec, plan):
    """dx = conv(dy, flip(W)^T) with pads K-1-p (stride 1)."""
    TD, TH, TW = plan
    geom = [spec.N, spec.OD, spec.OH, spec.OW, spec.K, spec.D, spec.H, spec.W, spec.KD, spec.KH, spec.KW,
            spec.KD - 1 - spec.pd, spec.KH - 1 - spec.ph, spec.KW - 1 - spec.pw, TD, TH, TW]
    wmat = halo_pack(w, spec, dgrad=True)                                    # [C][K/cs][Tp][cs], taps reversed
    dx = torch.empty(spec.N, spec.D, spec.H, spec.W, spec.C, dtype=torch.bfloat16, device=dy5.device)
    _halo_call(dy5, wmat, None, dx, None, geom, spec.C, 0)
    return dx


# ---------------------------------------------------------------------------
# raw native calls
# ---------------------------------------------------------------------------
def native_conv_fwd(x5: torch.Tensor, wmat: torch.Tensor, ldw: int, bias, spec: ConvSpec, act: int,
                    want_stats: bool, w: torch.Tensor | None = None, dstash: dict | None = None, pro=None):
    """``pro`` = ``bnfuse.pending(x5)``: x5 is a deferred BN output -- the tile kernel's prologue
    writes it from (y, prm) while it convolves, any other kernel has it written first."""
    # the tile kernel's epilogue has the identity and relu only
    tplan = conv_tile.fwd_plan(spec) if w is not None and act in (0, act_code("relu")) else None
    plan = halo_fwd_plan(spec) if w is not None else None
    # (``w`` may have fewer channels than spec: the halo packing zero-fills them itself, the tile
    # kernel takes the padded weight)
    if tplan is not None and (plan is None or conv_tile.choose(
            "fwd", spec, lambda: conv_tile.conv_fwd(x5, pad_to_spec(w, spec), bias, spec, act, want_stats, tplan),
            lambda: halo_conv_fwd(x5, w, bias, spec, act, want_stats, plan))):
        # (z itself is written only when something will read it: ``pro[4]`` -- the weight gradient
        # normalises y itself where it can, ConvFn decides)
        r = conv_tile.conv_fwd(x5, pad_to_spec(w, spec), bias, spec, act, want_stats, tplan, dstash=dstash,
                               pro=pro and (pro[0], pro[1], pro[2], x5 if pro[4] else None, pro[3]))
        if pro is not None:
            bnfuse.settle(x5, True)
        return r
    if pro is not None:
        bnfuse.settle(x5, False)
    if plan is not None:
        return halo_conv_fwd(x5, w, bias, spec, act, want_stats, plan)
    K = _native.kernels()
    assert x5.is_contiguous() and x5.dtype == torch.bfloat16
    gm = gather_mode(spec)
    tab = _table(spec, "fwd", gm, x5.device)
    y = torch.empty(spec.out_shape5, dtype=torch.bfloat16, device=x5.device)
    stats = None
    if want_stats:
        nmb = K.igemm_fwd_mblocks(spec.M)
        stats = torch.empty(nmb, 2, spec.K, dtype=torch.float32, device=x5.device)
    _igemm_fwd_call(K, x5, wmat, bias, y, stats, tab, _geom_fwd(spec), spec.M, spec.K, kdim_gather(spec), ldw, gm,
                    act)
    return y, stats


def _igemm_fwd_call(K, src, wt, bias, out, stats, tab, geom, M, N, kdim, ldw, gm, act):
    """igemm_fwd, in its split-K form (fp32 partial slabs, one reduce launch) where few row
    blocks meet a deep reduction and no statistics are wanted (``fn_igemm_fwd_splits``)."""
    splits = 1 if stats is not None else int(K.igemm_fwd_splits(M, N, kdim))
    part = part_scratch(splits * M * N, src.device) if splits > 1 else None
    K.igemm_fwd(src.data_ptr(), wt.data_ptr(), _native.ptr(bias), out.data_ptr(), _native.ptr(stats), tab.data_ptr(),
                geom, M, N, kdim, ldw, gm, act, _native.stream(src), _native.ptr(part), splits,
                0 if part is None else part.numel())


def native_conv_dgrad(dy5: torch.Tensor, w: torch.Tensor, spec: ConvSpec, bn=None, wpk=None):
    """dx of the conv.  ``bn = (y, prm, act)`` (x was a BN+act output, :mod:`.bnfuse`): returns
    ``(dx, slab)`` where ``slab`` holds that BN's backward sums from the tile kernel's
    epilogue, or None when another kernel ran.  ``w`` may have fewer output channels than
    ``spec.K`` (channel-padded dy): zero rows, materialised only for the tile kernel (the halo
    and gather packings zero-fill them)."""
    if w.shape[0] != spec.K and conv_tile.dgrad_plan(spec) is not None:
        w = pad_to_spec(w, spec)
    if bn is not None:
        tplan = conv_tile.dgrad_plan(spec)
        plan = halo_dgrad_plan(spec)
        if tplan is not None:
            dy5 = dy5.contiguous()
            if plan is None or conv_tile.choose("dgrad", spec, lambda: conv_tile.conv_dgrad(dy5, w, spec, tplan),
                                                lambda: halo_conv_dgrad(dy5, w, spec, plan)):
                return conv_tile.conv_dgrad(dy5, w, spec, tplan, bn=bn, wpk=wpk)
        return native_conv_dgrad(dy5, w, spec, wpk=wpk), None
    tplan = conv_tile.dgrad_plan(spec)
    plan = halo_dgrad_plan(spec)
    if tplan is not None:
        dy5 = dy5.contiguous()
        if plan is None or conv_tile.choose("dgrad", spec, lambda: conv_tile.conv_dgrad(dy5, w, spec, tplan),
                                            lambda: halo_conv_dgrad(dy5, w, spec, plan)):
            return conv_tile.conv_dgrad(dy5, w, spec, tplan, wpk=wpk)
    if plan is not None:
        return halo_conv_dgrad(dy5.contiguous(), w, spec, plan)
    K = _native.kernels()
    if spec.sd > 1 or spec.sh > 1 or spec.sw > 1:
        ODu, OHu, OWu = _dgrad_src_dims(spec)
        up = torch.zeros(spec.N, ODu, OHu, OWu, spec.K, dtype=torch.bfloat16, device=dy5.device)
        up[:, :: spec.sd, :: spec.sh, :: spec.sw] = dy5
        dy5 = up
    dy5 = dy5.contiguous()
    vec = GM_VEC if spec.K % 8 == 0 else GM_SCALAR
    tab = _table(spec, "dgrad", vec == GM_VEC, dy5.device)
    # WT[ci][tap][co] = w[co][tap][ci] (one cast + transpose launch; missing rows of w are zeros)
    if w.is_cuda:
        wt, ldw = _native_pack(w, spec, 1)
    else:
        w = pad_to_spec(w, spec)
        wt = w.reshape(spec.K, spec.taps, spec.C).permute(2, 1, 0).reshape(spec.C, spec.taps * spec.K)
        wt, ldw = _pack_rows(wt)
    dx = torch.empty(spec.N, spec.D, spec.H, spec.W, spec.C, dtype=torch.bfloat16, device=dy5.device)
    M = spec.N * spec.D * spec.H * spec.W
    _igemm_fwd_call(K, dy5, wt, None, dx, None, tab, _geom_dgrad(spec), M, spec.C, spec.taps * spec.K, ldw, vec, 0)
    return dx


def wgrad_splits(spec: ConvSpec, target_blocks: int = 1024) -> int:
    col_tiles = math.ceil(spec.kdim / 256)
    co_tiles = math.ceil(spec.K / 64) if spec.K > 32 else 1
    s = max(1, math.ceil(target_blocks / (col_tiles * co_tiles)))
    return int(min(s, max(1, spec.M // 256)))


def wgrad_takes_prologue(spec: ConvSpec) -> bool:
    """:func:`native_conv_wgrad` of ``spec`` will run conv_wtile in a form that applies a BN prologue
    to x itself (decided without timing; False when only an autotune run could tell)."""
    wplan = conv_wtile.plan(spec)
    if wplan is None or not conv_wtile.prologue_ok(wplan):
        return False
    if halo_wgrad_plan(spec) is None or conv_wtile.mode() == "2":
        return True
    from . import tuning

    return tuning.predict("wgrad", spec) is True


def native_conv_wgrad(dy5: torch.Tensor, x5: torch.Tensor, spec: ConvSpec, out=None, wdot=None, pro=None):
    """fp32 dW [K, KD, KH, KW, C]; ``out`` (zeroed, contiguous, that shape) receives it in place
    where the kernel allows.  ``wdot`` (the fp32 weights): returns ``(dW, S partials or None)``
    -- the big-tile kernel's reduce also sums S = W . dW per input channel (see
    :func:`conv_wtile.conv_wgrad`); None where another kernel ran.  ``pro`` = (y, prm, act, fill):
    x5 is a BN output the forward never wrote -- conv_wtile normalises y's halos itself, any other
    kernel has ``fill()`` write x5 first."""
    plan = halo_wgrad_plan(spec)
    wplan = conv_wtile.plan(spec)
    if wplan is not None:
        dy5, x5 = dy5.contiguous(), x5.contiguous()
        use = plan is None or conv_wtile.choose(
            spec, lambda: conv_wtile.conv_wgrad(dy5, x5, spec, wplan), lambda: halo_conv_wgrad(dy5, x5, spec, plan))
        if use and pro is not None and conv_wtile.prologue_ok(wplan):
            return conv_wtile.conv_wgrad(dy5, pro[0], spec, wplan, out=out, wdot=wdot, pro=(pro[1], pro[2]))
        if pro is not None:
            pro[3]()
            pro = None
        if use:
            return conv_wtile.conv_wgrad(dy5, x5, spec, wplan, out=out, wdot=wdot)
    if pro is not None:
        pro[3]()
    if wdot is not None:
        return native_conv_wgrad(dy5, x5, spec, out=out), None
    if plan is not None:
        return halo_conv_wgrad(dy5.contiguous(), x5.contiguous(), spec, plan, out=out)
    K = _native.kernels()
    gm = gather_mode(spec)
    if gm == GM_PACKW:                   # (the epilogue drops the packed rows' padding columns)
        dw = igemm_wgrad_cropped(dy5, x5, spec, spec.C, out=out)
        if dw is not None:
            return dw
    tab = _table(spec, "fwd", gm, x5.device)
    splits = wgrad_splits(spec)
    kd = kdim_gather(spec)
    # the kernel accumulates with atomics into a zeroed buffer: the flat gradient slice itself
    # (``out``, zeroed by FlatParams) when the layouts agree
    direct = (out is not None and gm != GM_PACKW and out.dtype == torch.float32 and out.is_contiguous()
              and out.numel() == spec.K * kd)
    dw = out.view(spec.K, kd) if direct else torch.zeros(spec.K, kd, dtype=torch.float32, device=x5.device)
    part = part_scratch(int(K.igemm_wgrad_part(spec.K, kd, splits, 0, 0, 0, 0)), x5.device)
    K.igemm_wgrad(dy5.data_ptr(), x5.data_ptr(), dw.data_ptr(), tab.data_ptr(), _geom_fwd(spec), spec.M, spec.K,
                  kd, splits, gm, _native.stream(x5), 0, 0, 0, 0, 0, 0, part.data_ptr(), part.numel())
    if direct:
        return out
    if gm == GM_PACKW:
        dw = dw.reshape(spec.K, spec.KD * spec.KH, -1)[:, :, : spec.KW * spec.C]
    dw = dw.reshape(spec.K, spec.KD, spec.KH, spec.KW, spec.C)
    if out is not None:
        return out.copy_(dw)
    return dw.contiguous()


def igemm_wgrad_takes(spec: ConvSpec) -> bool:
    """The weight gradient of ``spec`` (and of its 8-padded-Cout form) runs on the gather kernel
    (no halo / tile weight-gradient plan)."""
    sk = dataclasses.replace(spec, K=-(-spec.K // 8) * 8)
    return all(p is None for p in (halo_wgrad_plan(spec), conv_wtile.plan(spec), halo_wgrad_plan(sk),
                                   conv_wtile.plan(sk)))


def igemm_wgrad_cropped(dy5: torch.Tensor, x5: torch.Tensor, spec: ConvSpec, c0: int, out=None, ya=None,
                        act: int = 0, bias_param=None, with_db: bool = False):
    """fp32 dW [K, KD, KH, KW, c0] on the gather kernel, accumulated straight into ``out``
    (zeroed, e.g. the parameter's flat gradient) with every padding column of the gather
    layout dropped in the epilogue: the zero channels c0..spec.C of a channel-padded input,
    or the row padding of the packed-W layout (C < 8: rows of KW*C rounded up to 8).
    ``dy5`` has the real ``spec.K`` channels (padded here to a multiple of 8 for the kernel's
    16-B loads; the epilogue drops the padded rows).  ``ya`` / ``act``: dy5
    is the gradient of the activation output ``ya`` (the activation backward runs as dy is
    loaded); ``with_db``: the bias gradient from the same dy tiles too, into ``bias_param``'s
    zeroed flat-gradient slot when it offers one -- returns ``(dW, db)`` then.  None when the
    shape belongs to another weight-gradient kernel."""
    if not igemm_wgrad_takes(spec):
        return None
    gm = gather_mode(spec)
    if spec.C < c0:
        return None
    if gm == GM_PACKW:
        if c0 != spec.C:
            return None
        cpad, ccrop = packw_row(spec), spec.KW * spec.C   # row r*R + p -> r*KW*C + p, p < KW*C
    else:
        cpad, ccrop = spec.C, c0                          # tap t*C + c -> t*c0 + c, c < c0
    kd = kdim_gather(spec)
    if kd % cpad:
        return None
    shape = (spec.K, spec.KD, spec.KH, spec.KW, c0)
    if out is None or out.dtype != torch.float32 or not out.is_contiguous() or tuple(out.shape) != shape:
        out = torch.zeros(shape, dtype=torch.float32, device=x5.device)
    tab = _table(spec, "fwd", gm, x5.device)
    dy5, x5 = dy5.contiguous(), x5.contiguous()
    if ya is not None:
        ya = ya.contiguous()
        assert ya.dtype == torch.bfloat16 and ya.numel() == dy5.numel()
    kp = -(-spec.K // 8) * 8
    if kp != spec.K:
        # Cout % 8 != 0: dy channel-padded for 16-B row loads (single-element loads made this
        # kernel 1.45x slower on LeNet's 6-channel conv1), rows past K dropped by the epilogue
        if ya is not None:
            dy5, ya = native_act_bwd(dy5, ya, act), None
        dy5 = pad_channels(dy5, kp)
    db = _zeroed_grad(bias_param, spec.K, x5.device) if with_db else None
    K = _native.kernels()
    splits = wgrad_splits(spec)
    part = part_scratch(int(K.igemm_wgrad_part(kp, kd, splits, ccrop, cpad, spec.K, int(db is not None))), x5.device)
    K.igemm_wgrad(dy5.data_ptr(), x5.data_ptr(), out.data_ptr(), tab.data_ptr(), _geom_fwd(spec), spec.M, kp, kd,
                  splits, gm, _native.stream(x5), ccrop, cpad, _native.ptr(ya), act if ya is not None else 0,
                  _native.ptr(db), spec.K, part.data_ptr(), part.numel())
    return (out, db) if with_db else out


def bn_wdot(w: torch.Tensor, dw: torch.Tensor, spec: ConvSpec) -> torch.Tensor:
    """Per-block partial sums [nb, C] of sum_{k,t} bf16(W[k,t,c]) * dW[k,t,c] (fp32 weights and
    weight gradient of a conv over C input channels; ``bn_pool.hip`` bn_wdot_kernel)."""
    C = w.shape[-1]
    R = w.numel() // C
    w2 = w.float().contiguous()
    nb = int(max(1, min(64, -(-R // (256 // C)))))
    part = torch.empty(nb, C, dtype=torch.float32, device=w.device)
    _native.kernels().bn_wdot(w2.data_ptr(), dw.data_ptr(), part.data_ptr(), R, C, nb, _native.stream(w2),
                              [w2.numel(), dw.numel(), part.numel()])
    return part


def native_colsum(x2: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """Per-column sum of a [M, C] bf16 tensor in fp32 (bias gradients); into ``out`` (fp32
    [C], e.g. the bias's flat gradient slice) when given."""
    K = _native.kernels()
    M, C = x2.shape
    nb = int(max(1, min(1024, M // 64)))
    part = torch.empty(nb, 2, C, dtype=torch.float32, device=x2.device)
    st = _native.stream(x2)
    K.colstats(x2.data_ptr(), 0, 0, 0, 0, 0, part.data_ptr(), M, C, 0, 0, nb, st)
    tmp = torch.empty(2 if out is None else 1, C, dtype=torch.float32, device=x2.device)
    if out is not None:
        assert out.dtype == torch.float32 and out.is_contiguous() and out.numel() == C
    o0 = out if out is not None else tmp[0]
    K.bn_finalize(part.data_ptr(), nb, C, float(M), 0, 0, 0, 0, 0.0, 0.0, o0.data_ptr(), tmp[-1].data_ptr(), 0, 0,
                  1, st)
    return o0


def native_act_bwd(dy: torch.Tensor, y: torch.Tensor, act: int) -> torch.Tensor:
    if act == 0:
        return dy
    dx = torch.empty_like(dy)
    _native.kernels().act_bwd(dy.data_ptr(), y.data_ptr(), dx.data_ptr(), dy.numel(), act, _native.stream(dy))
    return dx


# ---------------------------------------------------------------------------
# autograd
# ---------------------------------------------------------------------------
# ---------------------------------------------------------------------------
# space-to-depth: strided convs with few input channels (FeatureNet-3D's
# 1-channel 7^3 stride-2 stem) become stride-1 convs with s^3*C channels
# ---------------------------------------------------------------------------
def s2d_plan(spec: ConvSpec):
    """(factors, ConvSpec') when a strided, few-channel conv maps onto the stride-1 halo
    kernels after a space-to-depth of the (zero-padded) input; else None.  Padding
    ("same") is folded into the packing: the packed grid covers the padded input, and
    the stride-1 conv over it is unpadded.

    The packed input has ``s^3*C`` real channels, zero-padded to 8 (one 8-channel
    halo slice, k-step = 4 taps x 8 channels) or 16; FeatureNet-3D's 1-channel
    7^3 stride-2 stem becomes a 4^3-tap conv over 8 channels (K = 512 vs the
    real 343)."""
    f = (spec.sd, spec.sh, spec.sw)
    if not _halo_enabled() or f == (1, 1, 1) or (spec.dd, spec.dh, spec.dw) != (1, 1, 1):
        return None
    cs = spec.C * f[0] * f[1] * f[2]
    if cs > 16:
        return None
    co = 8 if cs <= 8 else 16
    padded = (spec.D + spec.pd + spec.pads_hi[0], spec.H + spec.ph + spec.pads_hi[1], spec.W + spec.pw + spec.pads_hi[2])
    D2, H2, W2 = (-(-d // s) for d, s in zip(padded, f))
    k2 = tuple(-(-k // s) for k, s in zip((spec.KD, spec.KH, spec.KW), f))
    if k2[0] * k2[1] * k2[2] < 8 or D2 < k2[0] or H2 < k2[1] or W2 < k2[2]:
        return None
    spec2 = ConvSpec.make((spec.N, D2, H2, W2, co), spec.K, k2, 1, "valid")
    if (spec2.OD, spec2.OH, spec2.OW) != (spec.OD, spec.OH, spec.OW) or halo_fwd_plan(spec2) is None:
        return None
    return f, spec2


def s2d_input(x5: torch.Tensor, f, spec2: ConvSpec, pads=(0, 0, 0)) -> torch.Tensor:
    """Space-to-depth packed input [N, D2, H2, W2, C'] of x zero-padded by ``pads`` in front
    (``s2d_pack`` kernel on GPU)."""
    N, D, H, W, C = x5.shape
    sd, sh, sw = f
    pd, ph, pw = pads
    D2, H2, W2 = spec2.D, spec2.H, spec2.W
    if x5.is_cuda and _native.kernels_available():
        u8 = x5.dtype == torch.uint8              # (binary voxels as bytes: converted as they are read)
        x5 = x5.contiguous() if u8 else x5.to(torch.bfloat16).contiguous()
        out = torch.empty(N, D2, H2, W2, spec2.C, dtype=torch.bfloat16, device=x5.device)
        _native.kernels().s2d_pack(x5.data_ptr(), out.data_ptr(),
                                   [N, D, H, W, C, sd, sh, sw, D2, H2, W2, spec2.C, pd, ph, pw], _native.stream(x5),
                                   int(u8))
        return out
    xp = torch.zeros(N, D2 * sd, H2 * sh, W2 * sw, C, dtype=x5.dtype, device=x5.device)
    xp[:, pd:pd + D, ph:ph + H, pw:pw + W] = x5[:, :D2 * sd - pd, :H2 * sh - ph, :W2 * sw - pw]
    x2 = xp.view(N, D2, sd, H2, sh, W2, sw, C).permute(0, 1, 3, 5, 2, 4, 6, 7).reshape(N, D2, H2, W2, -1)
    out = torch.zeros(N, D2, H2, W2, spec2.C, dtype=x5.dtype, device=x5.device)
    out[..., : x2.shape[-1]] = x2
    return out


def _s2d_wgeom(w_shape, f, spec2: ConvSpec) -> list[int]:
    K, KD, KH, KW, C = w_shape
    return [K, KD, KH, KW, C, *f, spec2.KD, spec2.KH, spec2.KW, spec2.C]


def s2d_weight(w: torch.Tensor, f, spec: ConvSpec, spec2: ConvSpec) -> torch.Tensor:
    K, KD, KH, KW, C = w.shape
    sd, sh, sw = f
    kd, kh, kw = spec2.KD, spec2.KH, spec2.KW
    if w.is_cuda and _native.kernels_available():   # one launch (pad + permute + channel pad)
        wf = w.float().contiguous()
        out = torch.empty(K, kd, kh, kw, spec2.C, dtype=torch.float32, device=w.device)
        _native.kernels().s2d_weight_map(wf.data_ptr(), out.data_ptr(), _s2d_wgeom(w.shape, f, spec2), 0,
                                         _native.stream(wf), [wf.numel(), out.numel()])
        return out.to(w.dtype)
    wp = torch.zeros(K, kd * sd, kh * sh, kw * sw, C, dtype=w.dtype, device=w.device)
    wp[:, :KD, :KH, :KW] = w
    w2 = wp.view(K, kd, sd, kh, sh, kw, sw, C).permute(0, 1, 3, 5, 2, 4, 6, 7).reshape(K, kd, kh, kw, -1)
    out = torch.zeros(K, kd, kh, kw, spec2.C, dtype=w.dtype, device=w.device)
    out[..., : w2.shape[-1]] = w2
    return out


def s2d_weight_grad(dw2: torch.Tensor, f, spec: ConvSpec, out=None) -> torch.Tensor:
    """Inverse of :func:`s2d_weight` for a gradient (drops padded taps / channels); into
    ``out`` (fp32, the strided conv's weight shape, e.g. its flat gradient) when given."""
    K, kd, kh, kw, _ = dw2.shape
    sd, sh, sw = f
    C = spec.C
    if dw2.is_cuda and _native.kernels_available():
        src = dw2.float().contiguous()
        if out is None:
            out = torch.empty(K, spec.KD, spec.KH, spec.KW, C, dtype=torch.float32, device=dw2.device)
        _native.kernels().s2d_weight_map(src.data_ptr(), out.data_ptr(),
                                         [K, spec.KD, spec.KH, spec.KW, C, sd, sh, sw, kd, kh, kw, dw2.shape[-1]], 1,
                                         _native.stream(src), [src.numel(), out.numel()])
        return out
    g = dw2[..., : sd * sh * sw * C].reshape(K, kd, kh, kw, sd, sh, sw, C)
    g = g.permute(0, 1, 4, 2, 5, 3, 6, 7).reshape(K, kd * sd, kh * sh, kw * sw, C)
    return g[:, : spec.KD, : spec.KH, : spec.KW].contiguous()


def pointwise_ok(spec: ConvSpec, want_stats: bool = False) -> bool:
    """1x1x1 stride-1 unpadded conv that the streaming pointwise kernels take (pointwise.hip)."""
    return (spec.taps == 1 and (spec.sd, spec.sh, spec.sw) == (1, 1, 1) and not want_stats
            and (spec.pd, spec.ph, spec.pw) == (0, 0, 0) and spec.K <= 64 and spec.C <= 64
            and spec.M % 8 == 0 and spec.M >= 8)


def pw_fwd(x2: torch.Tensor, w2: torch.Tensor, bias, act: int, pro=None) -> torch.Tensor:
    """[M, Kin] x [Nout, Kin]^T (+bias, act) -> bf16 [M, Nout] on the pointwise kernel.

    ``pro = (scale, shift, act)``: the kernel reads ``act(x * scale + shift)`` (per input
    channel) instead of x -- a BN + activation that is never written to memory."""
    M, Kin = x2.shape
    N = w2.shape[0]
    if act and bias is None:
        bias = torch.zeros(N, dtype=torch.float32, device=x2.device)
    y = torch.empty(M, N, dtype=torch.bfloat16, device=x2.device)
    wb = w2.detach().to(torch.bfloat16).contiguous()
    psc, psh, pact = pro if pro is not None else (None, None, 0)
    _native.kernels().pw_fwd(x2.data_ptr(), wb.data_ptr(), _native.ptr(bias), y.data_ptr(), M, Kin, N, act,
                             _native.stream(x2), _native.ptr(psc), _native.ptr(psh), pact)
    return y


def pw_prologue_ok(K: int) -> bool:
    """Input channel counts the pointwise kernels' BN+act prologue supports."""
    return K % 8 == 0 and 2048 % K == 0


def pw_wgrad(dy2: torch.Tensor, x2: torch.Tensor, pro=None, out=None) -> torch.Tensor:
    """fp32 dW [Nout, Kin] = dy^T x on the pointwise kernel (``pro``: as :func:`pw_fwd`); into
    ``out`` (zeroed fp32 of N*Kin elements, e.g. the weight's flat gradient slice) when given."""
    M, N = dy2.shape
    Kin = x2.shape[1]
    if out is not None and out.is_contiguous() and out.dtype == torch.float32 and out.numel() == N * Kin:
        dw = out.view(N, Kin)
    else:
        dw = torch.zeros(N, Kin, dtype=torch.float32, device=x2.device)
    psc, psh, pact = pro if pro is not None else (None, None, 0)
    K = _native.kernels()
    part = part_scratch(int(K.pw_wgrad_blocks(M, Kin, N)) * N * Kin, x2.device)
    K.pw_wgrad(dy2.data_ptr(), x2.data_ptr(), dw.data_ptr(), M, Kin, N, _native.stream(x2), _native.ptr(psc),
               _native.ptr(psh), pact, part.data_ptr(), part.numel())
    return dw


# ---------------------------------------------------------------------------
# channel padding for NAS channel counts (C or Cout % 8 != 0)
# ---------------------------------------------------------------------------
def chan_pad_needed(spec: ConvSpec) -> bool:
    """The forward / wgrad gather would fall back to single-element loads (GM_SCALAR)."""
    return gather_mode(spec) == GM_SCALAR


def pad_channels(x: torch.Tensor, cp: int) -> torch.Tensor:
    """bf16 channels-last copy of ``x`` with its channels zero-padded to ``cp`` (one native pass)."""
    C = x.shape[-1]
    if C == cp:
        return x
    x = x.contiguous()
    out = torch.empty(*x.shape[:-1], cp, dtype=torch.bfloat16, device=x.device)
    _native.kernels().pad_channels(x.data_ptr(), out.data_ptr(), x.numel() // C, C, cp, 0, _native.stream(x),
                                   [x.numel(), out.numel()])
    return out


def pad_weight(w: torch.Tensor, cin: int | None = None, cout: int | None = None) -> torch.Tensor:
    """Zero-pad a [K, KD, KH, KW, C] weight to ``cout`` rows / ``cin`` input channels."""
    K, C = w.shape[0], w.shape[-1]
    pc, pk = (cin or C) - C, (cout or K) - K
    if pc == 0 and pk == 0:
        return w
    return F.pad(w, (0, pc, 0, 0, 0, 0, 0, 0, 0, pk))


def _zeroed_grad(p, n: int, device) -> torch.Tensor:
    """The parameter's zeroed flat-gradient slot, or a zeroed fp32 buffer of ``n``."""
    t = grad_target(p)
    return t if t is not None else torch.zeros(n, dtype=torch.float32, device=device)


def _conv_bwd_padded(ctx, dy, xs, w, spec, y=None):
    """ConvFn backward for channel-padded convs: ``xs`` is the (possibly channel-padded)
    saved input, ``spec`` its spec; dy (already through the activation backward) is padded
    to a multiple of 8 output channels when Cout % 8 != 0, the weight gets matching zero
    rows / columns, and the gradients are cropped back to the real channels.  ``y`` (the
    activation output, first layers only): dy is still pre-activation-backward, and the gather
    weight-gradient kernel applies it (and sums the bias gradient) as it loads dy."""
    C0 = w.shape[-1]
    K0 = spec.K
    kp = -(-K0 // 8) * 8
    sk = dataclasses.replace(spec, K=kp)
    dyp = None
    dx = dw = db = None
    if ctx.x_needs:                                              # real input channels: dx has C0 columns
        dyp = pad_channels(dy, kp)
        dx = native_conv_dgrad(dyp, w.detach(), dataclasses.replace(sk, C=C0))   # (zero rows K0..kp)
    want_db = ctx.has_b and ctx.needs_input_grad[2]
    if y is not None and not ctx.needs_input_grad[1]:
        dy, y = native_act_bwd(dy, y, ctx.act), None
    if ctx.needs_input_grad[1]:
        tgt = grad_target(w)
        if y is not None and not (kp != K0 or spec.C != C0):
            dy, y = native_act_bwd(dy, y, ctx.act), None
        if kp != K0 or spec.C != C0:
            # the gather kernel drops the padded channels itself and reads the unpadded dy
            r = igemm_wgrad_cropped(dy, xs, spec, C0, out=tgt, ya=y, act=ctx.act if y is not None else 0,
                                    bias_param=ctx.bparam, with_db=want_db)
            if r is not None:
                dw, db = r if want_db else (r, None)
            if dw is None:
                if y is not None:                # (the fused activation backward did not run)
                    dy = native_act_bwd(dy, y, ctx.act)
                    y = None
                dyp = pad_channels(dy, kp) if dyp is None else dyp
                dwp = native_conv_wgrad(dyp, xs.contiguous(), sk)     # [kp, KD, KH, KW, spec.C]
                dw = tgt.copy_(dwp[:K0, ..., :C0]) if tgt is not None else dwp[:K0, ..., :C0].contiguous()
        else:
            dyp = pad_channels(dy, kp) if dyp is None else dyp
            dw = native_conv_wgrad(dyp, xs.contiguous(), sk, out=tgt)
    if want_db and db is None:
        db = native_colsum(dy.reshape(-1, K0), out=grad_target(ctx.bparam))
    return dx, dw, db, None, None, None


def _stashed(ctx):
    """The dgrad's packed weights the forward made (conv_tile.conv_fwd ``dstash``), or None;
    released once taken."""
    st = getattr(ctx, "dstash", None)
    ctx.dstash = None
    return st.get("wpk") if st else None


class ConvFn(torch.autograd.Function):
    """y = act(conv(x, w) + b); optional BN statistics slab as a 2nd output."""

    @staticmethod
    def forward(ctx, x5, w, b, spec: ConvSpec, act: int, want_stats: bool):
        w0 = w
        bias = b.detach().float().contiguous() if b is not None else None
        s2d = s2d_plan(spec)
        x_saved = x5
        ctx.pw = pointwise_ok(spec, want_stats)
        ctx.cpad = 0
        # x = a deferred BN output (ops/bnfuse.py): the tile forward writes it; every other branch
        # has it written before reading it
        pro = bnfuse.pending(x5)
        tile_branch = (not ctx.pw and s2d is None and not chan_pad_needed(spec) and
                       (halo_fwd_plan(spec) is not None or
                        (conv_tile.fwd_plan(spec) is not None and act in (0, act_code("relu")))))
        if pro is not None and not tile_branch:
            bnfuse.settle(x5, False)
            pro = None
        ctx.pro_w = None                 # (y, prm, act, fill): the backward's wgrad normalises y itself
        if pro is not None:
            # z is read by nothing but this conv's weight gradient
            zw = bool(ctx.needs_input_grad[1]) and not (bnfuse.prologue_wgrad_enabled() and
                                                        wgrad_takes_prologue(spec))
            if ctx.needs_input_grad[1] and not zw:
                ctx.pro_w = (pro[0], pro[1], pro[2], bnfuse.filler(x5))
            pro = pro + (zw,)
        if not ctx.pw and s2d is None and chan_pad_needed(spec):
            # C % 8 != 0 (NAS convs: 12, 18, 120 ... channels): gather 16-B channel vectors of a
            # zero-padded copy instead of single elements; the padded copy is what wgrad reads
            cp = -(-spec.C // 8) * 8
            x5 = pad_channels(x5, cp)
            spec = dataclasses.replace(spec, C=cp)              # (w keeps its C0 channels: zero-padded
            #                                                     by the packing or pad_to_spec below)
            x_saved = x5
            ctx.cpad = cp
        if ctx.pw:
            x5 = x5.contiguous()
            y = pw_fwd(x5.reshape(-1, spec.C), w.reshape(spec.K, spec.C), bias, act).reshape(spec.out_shape5)
            stats = None
            s2d = None
            x_saved = x5
        elif s2d is not None and s2d[1].kdim <= S2D_FWD_RATIO * spec.kdim:
            # strided few-channel conv: space-to-depth -> stride-1 halo conv; the packed
            # input is what wgrad consumes, so it is saved instead of x
            f, spec2 = s2d
            x2 = s2d_input(x5, f, spec2, (spec.pd, spec.ph, spec.pw))
            y, stats = native_conv_fwd(x2, None, 0, bias, spec2, act, want_stats,
                                       w=s2d_weight(w.detach(), f, spec, spec2))
            x_saved = x2
        elif s2d is not None:
            # the padded s2d K (FeatureNet-3D stem: 512 vs 343) loses to the packed-W gather
            # forward; wgrad still runs on the packed input
            f, spec2 = s2d
            wmat, ldw = pack_weight_rows(w.detach(), spec)
            y, stats = native_conv_fwd(x5.contiguous(), wmat, ldw, bias, spec, act, want_stats)
            x_saved = s2d_input(x5, f, spec2, (spec.pd, spec.ph, spec.pw)) if ctx.needs_input_grad[1] else x5
        elif halo_fwd_plan(spec) is not None or (conv_tile.fwd_plan(spec) is not None and act in (0, act_code("relu"))):
            # (the tile forward also packs the backward's dgrad weights, in the same launch)
            ctx.dstash = {} if ctx.needs_input_grad[0] else None
            y, stats = native_conv_fwd(x5.contiguous(), None, 0, bias, spec, act, want_stats,
                                       w=w.detach(), dstash=ctx.dstash, pro=pro)
        else:
            wmat, ldw = pack_weight_rows(w.detach(), spec)
            y, stats = native_conv_fwd(x5.contiguous(), wmat, ldw, bias, spec, act, want_stats)
        ctx.spec, ctx.act, ctx.has_b, ctx.s2d = spec, act, b is not None, s2d   # (channel-padded spec when cpad)
        ctx.pack_gen = _PK_TLS.gen                      # (the backward's packs: this forward's scope)
        ctx.bparam = b
        ctx.set_materialize_grads(False)                # no zero-filled gradient for the stats output
        ctx.x_needs = ctx.needs_input_grad[0]
        # x = act(bn(y)) of the previous layer: the dgrad epilogue sums that BN's backward
        # statistics (ops/bnfuse.py) -- plain stride-1 convs on the tile kernel only
        ctx.bn_src = (bnfuse.source_of(x_saved) if ctx.x_needs and not ctx.pw and s2d is None and
                      conv_tile.dgrad_plan(spec) is not None else None)
        ctx.save_for_backward(x_saved, w0, y if act else None)
        if stats is not None:
            ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    def backward(ctx, dy, _dstats):
        if dy is None:
            return None, None, None, None, None, None
        with packs.gen_as(ctx.pack_gen):
            return ConvFn._backward(ctx, dy)

    @staticmethod
    def _backward(ctx, dy):
        x5, w, y = ctx.saved_tensors
        spec, act = ctx.spec, ctx.act
        dy = dy.contiguous().to(torch.bfloat16)
        padded = ctx.cpad or (spec.K % 8 and ctx.s2d is None)
        # the gather weight-gradient kernel is dy's only consumer (no input gradient: a first
        # layer): it applies the activation backward and sums the bias gradient as it loads dy
        wg_igemm = (not ctx.pw and ctx.s2d is None and ctx.needs_input_grad[1] and igemm_wgrad_takes(spec)
                    and (not padded or ctx.cpad or spec.C == w.shape[-1]))
        # x5 unwritten (the forward's BN prologue): native_conv_wgrad's conv_wtile normalises y
        # itself; any other weight-gradient path has x5 written first
        prow, ctx.pro_w = getattr(ctx, "pro_w", None), None
        if prow is not None and (padded or ctx.pw or ctx.s2d is not None or wg_igemm):
            prow[3]()
            prow = None
        fuse_act = bool(act) and wg_igemm and not ctx.x_needs
        if act and not fuse_act:
            dy = native_act_bwd(dy, y, act)
        if padded:
            return _conv_bwd_padded(ctx, dy, x5, w, spec, y=y if fuse_act else None)
        if ctx.pw:
            dy2, x2 = dy.reshape(-1, spec.K), x5.reshape(-1, spec.C)
            dx = pw_fwd(dy2, w.detach().reshape(spec.K, spec.C).t(), None, 0).reshape(x5.shape) if ctx.x_needs else None
            dw = pw_wgrad(dy2, x2, out=grad_target(w)).reshape(w.shape) if ctx.needs_input_grad[1] else None
            db = native_colsum(dy2, out=grad_target(ctx.bparam)) if (ctx.has_b and ctx.needs_input_grad[2]) else None
            return dx, dw, db, None, None, None
        dx = None
        ident = None                     # the statistics identity's sum-g slab (bnfuse)
        bn_y = None
        if ctx.x_needs:
            if ctx.bn_src is not None:
                bn_y = ctx.bn_src[0]
                dx, slab = native_conv_dgrad(dy, w.detach(), spec, bn=ctx.bn_src, wpk=_stashed(ctx))
                if isinstance(slab, tuple):
                    ident = slab[1]              # (offered below, with S from this conv's dW)
                ctx.bn_src = None
            else:
                dx = native_conv_dgrad(dy, w.detach(), spec, wpk=_stashed(ctx))
        dw = db = None
        wpart = None
        want_db = ctx.has_b and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1]:
            if ctx.s2d is not None:      # x5 is the space-to-depth packed input (saved by forward)
                f, spec2 = ctx.s2d
                dw = s2d_weight_grad(native_conv_wgrad(dy, x5, spec2), f, spec, out=grad_target(w))
            elif wg_igemm:               # (+ the bias gradient, + the activation backward if fused)
                tgt = grad_target(w)
                r = igemm_wgrad_cropped(dy, x5, spec, spec.C, out=tgt, ya=y if fuse_act else None,
                                        act=act if fuse_act else 0, bias_param=ctx.bparam, with_db=want_db)
                if r is not None:
                    dw, db = r if want_db else (r, None)
                else:                    # (not taken after all: the separate passes)
                    if fuse_act:
                        dy = native_act_bwd(dy, y, act)
                    dw = native_conv_wgrad(dy, x5.contiguous(), spec, out=tgt)
            elif ident is not None and w.dtype == torch.float32:
                # (+ S = sum W . dW for the statistics identity from the reduce pass, when it can)
                dw, wpart = native_conv_wgrad(dy, x5.contiguous(), spec, out=grad_target(w), wdot=w.detach(),
                                              pro=prow)
            else:
                # straight into the parameter's zeroed flat gradient when FlatParams offers it
                dw = native_conv_wgrad(dy, x5.contiguous(), spec, out=grad_target(w), pro=prow)
        if want_db and db is None:
            db = native_colsum(dy.reshape(-1, spec.K), out=grad_target(ctx.bparam))
        if ident is not None:
            if dw is not None and dw.dtype == torch.float32 and dw.is_contiguous() and dw.numel() == w.numel():
                # S = sum W . dW per input channel, read before any data-parallel all-reduce of dW
                # (its hook fires after this backward returns)
                if wpart is None:
                    wpart = bn_wdot(w.detach(), dw, spec)
                bnfuse.offer(dx, ("identity", ident, wpart), bn_y)
            # (else: no offer -- the BN backward's colstats pass reads the masked dx, which its
            # relu mask leaves unchanged)
        return dx, dw, db, None, None, None


def conv(x5: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None, spec: ConvSpec, act=None,
         want_stats: bool = False):
    """Convolution on a 5-D channels-last tensor.

    Returns ``y`` or ``(y, stats)`` when ``want_stats`` (GPU only; stats is the
    per-block (sum, sumsq) slab consumed by :func:`ops.bn.batchnorm_act`).
    """
    if _native.use_native(x5):
        # uint8 input (binary voxel occupancy) goes to the space-to-depth stem as is: its packing
        # kernel reads the bytes (a quarter of the bf16 traffic); every other conv takes bf16
        xin = x5 if x5.dtype == torch.uint8 and u8_input_ok(spec) else x5.to(torch.bfloat16)
        y, stats = ConvFn.apply(xin, w, b, spec, act_code(act), want_stats)
        return (y, stats) if want_stats else y
    if not x5.is_floating_point():
        x5 = x5.to(w.dtype)                       # (uint8 voxels on the reference path)
    y = ref.conv(x5, w.to(x5.dtype), None if b is None else b.to(x5.dtype), spec, act)
    return (y, None) if want_stats else y


def u8_input_ok(spec: ConvSpec) -> bool:
    """The conv reads its input only through the space-to-depth packing (ConvFn's s2d branch):
    a uint8 input may be passed as is."""
    s2d = s2d_plan(spec)
    return s2d is not None and not pointwise_ok(spec) and s2d[1].kdim <= S2D_FWD_RATIO * spec.kdim


def _dw_geom(spec: ConvSpec) -> list[int]:
    return [spec.N, spec.D, spec.H, spec.W, spec.C, spec.OD, spec.OH, spec.OW, spec.KD, spec.KH, spec.KW,
            spec.sd, spec.sh, spec.sw, spec.pd, spec.ph, spec.pw, spec.dd, spec.dh, spec.dw]


class DepthwiseFn(torch.autograd.Function):
    """Depthwise conv (multiplier 1) on ``dwconv.hip``: y = act(dwconv(x, w) + b)."""

    @staticmethod
    def forward(ctx, x5, w, b, spec: ConvSpec, act: int):
        K = _native.kernels()
        x5 = x5.contiguous()
        wf = w.detach().float().reshape(spec.C, spec.taps).contiguous()
        bias = b.detach().float().contiguous() if b is not None else None
        y = torch.empty(spec.N, spec.OD, spec.OH, spec.OW, spec.C, dtype=torch.bfloat16, device=x5.device)
        K.dw_fwd(x5.data_ptr(), wf.data_ptr(), _native.ptr(bias), y.data_ptr(), _dw_geom(spec), act,
                 _native.stream(x5))
        ctx.spec, ctx.act, ctx.has_b = spec, act, b is not None
        ctx.wparam, ctx.bparam = w, b
        ctx.save_for_backward(x5, wf, y if act else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x5, wf, y = ctx.saved_tensors
        spec, act = ctx.spec, ctx.act
        K = _native.kernels()
        st = _native.stream(x5)
        dy = dy.contiguous().to(torch.bfloat16)
        if act:
            dy = native_act_bwd(dy, y, act)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x5)
            K.dw_dgrad(dy.data_ptr(), wf.data_ptr(), dx.data_ptr(), _dw_geom(spec), st)
        if ctx.needs_input_grad[1]:
            tgt = grad_target(ctx.wparam)           # (zeroed flat slice: the kernel accumulates)
            if tgt is not None and tgt.is_contiguous() and tgt.numel() == spec.C * spec.taps:
                dwf = tgt.view(spec.C, spec.taps)
            else:
                dwf = torch.zeros(spec.C, spec.taps, dtype=torch.float32, device=x5.device)
            splits = int(max(1, min(256, spec.M // 2048)))
            part = part_scratch(splits * spec.C * spec.taps, x5.device)
            K.dw_wgrad(dy.data_ptr(), x5.data_ptr(), dwf.data_ptr(), _dw_geom(spec), splits, st, part.data_ptr(),
                       part.numel())
            dw = tgt if dwf.data_ptr() == (tgt.data_ptr() if tgt is not None else -1) else \
                dwf.reshape(spec.C, spec.KD, spec.KH, spec.KW, 1)
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = native_colsum(dy.reshape(-1, spec.C), out=grad_target(ctx.bparam))
        return dx, dw, db, None, None


def depthwise_conv(x5: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None, spec: ConvSpec, mult: int = 1,
                   act=None) -> torch.Tensor:
    """Depthwise conv (reference ``DepthwiseConv2D`` / first half of ``SeparableConv2D``,
    ``model/input.py:296-306``): native ``dwconv.hip`` on GPU for depth multiplier 1
    (the only multiplier the reference search space produces); the PyTorch
    reference handles the CPU path and multipliers > 1.
    """
    if _native.use_native(x5) and mult == 1:
        return DepthwiseFn.apply(x5.to(torch.bfloat16), w, b, spec, act_code(act))
    dt = x5.dtype
    y = ref.depthwise_conv(x5.float() if x5.is_cuda else x5, w.float() if x5.is_cuda else w.to(dt),
                           None if b is None else (b.float() if x5.is_cuda else b.to(dt)), spec, mult, act)
    return y.to(dt)
