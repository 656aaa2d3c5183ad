"""Host side of the big-tile halo conv kernel (``csrc/kernels/conv_tile.hip``).

The kernel runs 4 waves per workgroup, one per SIMD, each owning ``16*MT``
output rows (512-640-row tiles), with the input halo of a ``CS``-channel
slice double-buffered in LDS (LDS-DMA) and the weights streamed from L2
straight into MFMA fragments.  This module

* plans the output tile (``TD x TH x TW``), the channel slice and ``MT`` for
  a layer from a simple cycle model (MFMA k-steps per job + per-job fixed
  cost, tail rounding over the 256 CUs), subject to the 160 KiB LDS;
* builds the row table that permutes the tile's output rows into MFMA
  fragments whose 16 rows have 16 distinct halo positions mod 16 -- with the
  chunk-planar halo layout that makes every ``ds_read_b128`` A-fragment read
  bank-conflict free;
* packs the conv weight into the fragment-ordered B stream (one HIP launch).

Reference parity: this is the same convolution as ``ops/conv.py`` (Keras
``Conv2D``/``Conv3D`` semantics, reference ``model/input.py:294``); only the
MI355X execution strategy differs.
"""
from __future__ import annotations

import math
import os
import threading
from dataclasses import dataclass

import numpy as np
import torch

from .. import _native
from . import packs

LDS_MAX = 160 * 1024
NTHR = 320          # 4 MFMA waves + 1 loader wave
MT_CHOICES = (8, 9)


def experiments_built() -> bool:
    """The kernel library was built with ``FN_BUILD_EXPERIMENTS=1`` (the int8 fp8-stem instance,
    the timing-only variants)."""
    try:
        return bool(_native.kernels().experiments_built())
    except Exception:                            # noqa: BLE001 - no library (CPU): nothing built
        return False


def red_bytes(NT: int, f8: bool = False) -> int:
    """LDS bytes of the per-compute-wave BN partial sums (4 waves x 2 x NT*16 columns: the running
    sums and the chunk flush rows of both job parities -- csrc conv_tile_shared.h ct_red_bytes)."""
    return (1 if f8 else 3) * 4 * 2 * NT * 16 * 4


_LOCK = threading.Lock()
_PLANS: dict = {}
_ROWTAB: dict = {}
_ZERO: dict = {}
_SCHED: dict = {}


def enabled() -> bool:
    return os.environ.get("FN_CONV_TILE", "1") != "0"


@dataclass(frozen=True)
class TilePlan:
    TD: int
    TH: int
    TW: int
    CS: int          # channels per halo slice
    MT: int          # 16-row MFMA tiles per wave
    NT: int          # 16-col MFMA tiles per workgroup (2: 32-column blocks)
    HPpad: int
    nks: int         # k-steps per job
    nct: int         # 16-col tiles of the packed weights
    BUF: int         # bytes per LDS buffer
    mHW: int
    mHHW: int
    cost: float      # modelled cycles (per wave, summed over the jobs of one CU)
    f8: bool = False  # fp8 (e4m3) inference variant: 16-channel chunks, 128-k steps, ring depth 2
    pool: bool = False  # fp8: fused 2^3 max-pool epilogue (even tile dims, window-per-lane row table)
    bs: bool = False    # fp8 with block-scaled activations: the block-scaled operand layout (k_table,
    #                     pack_weights_f8), two k-table rows per k-step, the LDS scale planes

    @property
    def rows(self) -> int:
        return self.TD * self.TH * self.TW


def _magic(d: int) -> int:
    return (2**32 + d - 1) // d


def _magic_ok(HH: int, HW: int, npos: int) -> bool:
    p = np.arange(npos, dtype=np.uint64)
    m2, m1 = np.uint64(_magic(HH * HW)), np.uint64(_magic(HW))
    hd = (p * m2) >> np.uint64(32)
    rem = p - hd * np.uint64(HH * HW)
    hh = (rem * m1) >> np.uint64(32)
    return bool(np.all(hd == p // np.uint64(HH * HW)) and np.all(hh == rem // np.uint64(HW)))


def _ksteps(T: int, CS: int, PD: int) -> int:
    k = T * (CS // 32) if CS >= 32 else -(-T // (32 // CS))   # CS = 16 / 8: 2 / 4 taps per k-step
    return -(-k // PD) * PD


def plan(N: int, out_dims: tuple, kdims: tuple, Csrc: int, Ncol: int, n_cus: int = 256, f8: bool = False,
         pool: bool = False, bs: bool = False, nt4: bool = False):
    """Best TilePlan for an (N, OD, OH, OW) output of a (KD, KH, KW) stride-1 conv over
    ``Csrc`` input channels into ``Ncol`` columns, or None when the kernel does not apply
    (``f8``: the e4m3 inference variant, 32- or 64-channel slices; ``pool``: with the fused
    2^3 max-pool epilogue -- even output and tile dims; ``bs``: block-scaled fp8 operands, the
    LDS also holds two planes of the halo positions' scale dwords; ``nt4``: 64-column workgroups
    over 256 rows (MT 4 x NT 4, bf16, Ncol % 64 == 0) -- one halo DMA for 64 columns instead of
    one per 32-column block, for loader-bound convs)."""
    bs = bool(bs and f8)
    nt4 = bool(nt4 and not f8 and Ncol % 64 == 0)
    key = (N, tuple(out_dims), tuple(kdims), Csrc, Ncol, n_cus, f8, pool, bs, nt4,
           os.environ.get("FN_TILE_PLAN_RANK", "0"))
    if key in _PLANS:
        return _PLANS[key]
    if pool and (not f8 or any(d % 2 for d in out_dims)):
        return None
    best = _plan(N, out_dims, kdims, Csrc, Ncol, n_cus, f8, pool, bs, nt4)
    with _LOCK:
        _PLANS[key] = best
    return best


def _plan(N, out_dims, kdims, Csrc, Ncol, n_cus, f8=False, pool=False, bs=False, nt4=False):
    OD, OH, OW = out_dims
    KD, KH, KW = kdims
    T = KD * KH * KW
    if Ncol < 16 or Ncol % 8 or Csrc % 8 or T < 2:
        return None
    NT = 4 if nt4 else 2                         # 32-column workgroups (nt4: 64, MT = 4)
    ncb = -(-Ncol // (NT * 16))
    nct = ncb * NT
    PD = PD_F8 if f8 else 4
    workers = max(1, n_cus // ncb)
    cands = []
    cs_only = int(os.environ.get("FN_TILE_CS", "0"))
    mt_choices = (8,) if f8 else ((4,) if nt4 else MT_CHOICES)
    for CS in ((64, 32) if f8 else ((32,) if nt4 else (32, 16, 8))):
        if Csrc % CS or (cs_only and CS != cs_only) or (CS == 8 and Csrc % 16 == 0):
            continue
        CPP = CS // 16 if f8 else CS // 8
        nslice = Csrc // CS
        nks = -(-math.ceil(T / (128 // CS)) // PD) * PD if f8 else _ksteps(T, CS, PD)   # f8: 128-k steps
        tw_opts = sorted({OW} | {-(-OW // k) for k in range(2, 5) if -(-OW // k) >= 8})
        for TW in tw_opts:
            for TD in range(1, OD + 1):
                for TH in range(1, OH + 1):
                    rows = TD * TH * TW
                    if rows > 64 * mt_choices[-1]:
                        break
                    if pool and (TD % 2 or TH % 2 or TW % 2):
                        continue
                    MT = max(mt_choices[0], -(-rows // 64))
                    if rows < 64 * mt_choices[0] * 0.75:
                        continue
                    HH, HW = TH + KH - 1, TW + KW - 1
                    HP = (TD + KD - 1) * HH * HW
                    HPpad = -(-HP // 64) * 64
                    BUF = HPpad * CPP * 16                     # the halo (a multiple of 2 KiB)
                    lds = 2 * BUF + 64 + red_bytes(NT, f8) + (nks + PD + 2) * 16 * (2 if bs else 1) + HPpad * 8 \
                        + (NT * 16 * 8 if f8 else 0) + (2 * HPpad * 4 if bs else 0)
                    if lds > LDS_MAX:
                        continue
                    tiles = N * -(-OD // TD) * -(-OH // TH) * -(-OW // TW)
                    jobs = tiles * nslice
                    mfma = nks * MT * NT * (32 if f8 else 16)  # cycles of MFMA issue per wave per job
                    fixed = 800                                 # barrier + first halo reads per job
                    epi = MT * NT * 40 / nslice                 # register epilogue, once per tile
                    loader = 1500 + (CPP * HPpad // 64) * 130   # DMA issue + landing of one job's halo
                    per_job = max(mfma + fixed + epi, loader)
                    cost = math.ceil(jobs / workers) * per_job
                    if bs and HP * 16 >= 65536:
                        continue                               # (packed 16-bit data offsets)
                    cands.append(TilePlan(TD, TH, TW, CS, MT, NT, HPpad, nks, nct, BUF, _magic(HW), _magic(HH * HW),
                                          float(cost), f8, pool, bs))
    # the cheapest few, re-costed with their row tables' residual bank conflicts (a
    # fragment whose 16 rows repeat a residue mod 16 reads at half rate).  (A finer term --
    # bank_ways, the simulated ways of every ds_read_b128 lane group -- was tried: conv4 fwd's
    # 2.1-way plan times equal to its conflict-free alternatives and the stem's conflict-free
    # plans need MT = 9, 7 % slower; profiles/r4_tile_plan_bank_sweep.md)
    ranked = []
    for c in sorted(cands, key=lambda c: c.cost)[:12]:
        HH, HW = c.TH + KH - 1, c.TW + KW - 1
        if not _magic_ok(HH, HW, c.HPpad):
            continue
        if f8:
            # fp8: the simulated ways of its reads (the parity tables below repeat residues by
            # design); the fused-pool conv4 went 2.8 -> 1.0 ways and 9 % faster
            cost = c.cost * (1.0 + 0.5 * (bank_ways(c, kdims) - 1.0))
        else:
            tab = row_table(c, kdims)
            res = tab[:, 0].reshape(-1, 16) % 16
            dups = sum(16 - len(set(r.tolist())) for r in res)
            cost = c.cost * (1.0 + 0.5 * dups / res.size)
        ranked.append(TilePlan(*(getattr(c, f) for f in ("TD", "TH", "TW", "CS", "MT", "NT", "HPpad", "nks", "nct",
                                                          "BUF", "mHW", "mHHW")), cost, f8, pool, bs))
    if not ranked:
        return None
    ranked.sort(key=lambda c: c.cost)
    # FN_TILE_PLAN_RANK=k: the k-th cheapest plan of the model (timing sweeps of the cost model)
    k = int(os.environ.get("FN_TILE_PLAN_RANK", "0"))
    return ranked[min(k, len(ranked) - 1)]


def row_table(p: TilePlan, kdims: tuple) -> np.ndarray:
    """int32 [4*MT*16, 2]: (halo position of the row's tap (0,0,0), natural tile row or -1),
    fragments of 16 rows with distinct halo positions mod 16 (bank-conflict-free A reads)."""
    key = (p, tuple(kdims))
    t = _ROWTAB.get(key)
    if t is not None:
        return t
    KD, KH, KW = kdims
    HH, HW = p.TH + KH - 1, p.TW + KW - 1
    if p.pool:
        tab = _pool_row_table(p, HH, HW)
        with _LOCK:
            _ROWTAB[key] = tab
        return tab
    tab = _std_row_table(p, HH, HW)
    if p.f8 and p.CS == 32:
        # fp8 32-channel slices read 4 taps per k-step, one per lane group, and a ds_read_b128
        # group mixes two lane groups: rows {0-3, 12-15} of one tap with rows {4-11} of the
        # next.  Distinct residues per fragment do not survive that shift; fragments of one
        # residue parity (each half holding all 8 residues of it) do, for every odd tap step.
        alt = _parity_row_table(p, HH, HW)
        if _table_ways(alt, p, kdims) < _table_ways(tab, p, kdims):
            tab = alt
    with _LOCK:
        _ROWTAB[key] = tab
    return tab


def _rows_and_positions(p: TilePlan, HH: int, HW: int):
    td, th, tw = np.meshgrid(np.arange(p.TD), np.arange(p.TH), np.arange(p.TW), indexing="ij")
    nat = ((td * p.TH + th) * p.TW + tw).reshape(-1)
    hb = ((td * HH + th) * HW + tw).reshape(-1)
    return nat, hb


def _fill_rest(frags: list, extra: list, maxhb: int) -> np.ndarray:
    for f in frags:                              # overflow rows fill free slots (a conflict, not an error)
        for s in range(16):
            if f[s] is None and extra:
                f[s] = extra.pop()
    assert not extra, "row table overflow"
    for f in frags:                              # dummies: a missing residue, inside the halo
        for s in range(16):
            if f[s] is None:
                used = {x[0] % 16 for x in f if x is not None}
                cand = [r for r in range(16) if r not in used and r <= maxhb]
                f[s] = ((cand[0] if cand else 0), -1)
    return np.asarray([x for f in frags for x in f], dtype=np.int32)


def _parity_row_table(p: TilePlan, HH: int, HW: int) -> np.ndarray:
    """Fragments of one residue parity: lanes {0-3, 12-15} and {4-11} each take one row of
    every residue of the fragment's parity (the parity with more rows left)."""
    nat, hb = _rows_and_positions(p, HH, HW)
    buckets = [list(zip(hb[hb % 16 == r].tolist(), nat[hb % 16 == r].tolist())) for r in range(16)]
    halves = ((0, 1, 2, 3, 12, 13, 14, 15), (4, 5, 6, 7, 8, 9, 10, 11))
    frags = []
    for _ in range(4 * p.MT):
        even = sum(len(buckets[r]) for r in range(0, 16, 2))
        odd = sum(len(buckets[r]) for r in range(1, 16, 2))
        par = 0 if even >= odd else 1
        f = [None] * 16
        for lanes in halves:
            for k, lr in enumerate(lanes):
                if buckets[par + 2 * k]:
                    f[lr] = buckets[par + 2 * k].pop()
        frags.append(f)
    return _fill_rest(frags, [x for b in buckets for x in b], int(hb.max()))


def _std_row_table(p: TilePlan, HH: int, HW: int) -> np.ndarray:
    nat, hb = _rows_and_positions(p, HH, HW)
    nfrag = 4 * p.MT
    buckets = [list(zip(hb[hb % 16 == r].tolist(), nat[hb % 16 == r].tolist())) for r in range(16)]
    frags = [[None] * 16 for _ in range(nfrag)]
    extra = []
    for r in range(16):
        for i, item in enumerate(buckets[r]):
            if i < nfrag:
                frags[i][r] = item
            else:
                extra.append(item)
    return _fill_rest(frags, extra, int(hb.max()))


# the lanes of each ds_read_b128 bank group (MI355X: four non-contiguous 16-lane groups)
_B128_GROUPS = np.array([[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
                         [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]])
_B128_GROUPS = np.concatenate([_B128_GROUPS, _B128_GROUPS + 32])
_WAYS: dict = {}


def bank_ways(p: TilePlan, kdims: tuple) -> float:
    """Mean ways of the kernel's halo-fragment reads (ds_read_b128: bank of byte address a is
    (a / 4) mod 64, so a lane's 16-B read takes slot (a / 16) mod 16) over every fragment, every
    distinct k-step tap pattern and the four lane groups the LDS serves together; 1.0 =
    conflict-free.  Lane l = (lane group lg = l / 16, fragment row lr = l % 16) reads halo
    position rowtab[lr] at the plane and tap offset of lg (``lb`` / ``s_kt`` in conv_tile.hip).
    The groups mix rows of two lane groups ({0-3, 12-15} of one with {4-11} of the next), so a
    k-step whose lane groups read different taps (CS = 8, fp8) shifts one half's residues."""
    key = (p, tuple(kdims))
    w = _WAYS.get(key)
    if w is None:
        w = _table_ways(row_table(p, kdims), p, kdims)
        with _LOCK:
            _WAYS[key] = w
    return w


def _table_ways(tab: np.ndarray, p: TilePlan, kdims: tuple) -> float:
    kt = k_table(p, kdims)[:p.nks]
    hb = tab[:, 0].reshape(-1, 16).astype(np.int64)               # [fragments, 16 rows]
    lg, lr = _B128_GROUPS // 16, _B128_GROUPS % 16                 # [4, 16]
    cpp = p.CS // 16 if p.f8 else p.CS // 8
    if p.f8:
        pl = 2 * (lg & 1) if cpp == 4 else 0 * lg
    else:
        pl = lg if cpp >= 4 else ((lg & 1) if cpp == 2 else 0 * lg)
    pats = np.unique(kt.astype(np.int64), axis=0)                  # distinct k-step offset rows
    a = hb[:, lr][:, None] * 16 + (pl * p.HPpad * 16)[None, None] + pats[:, lg][None]   # [F, P, 4, 16]
    a = np.sort(a, axis=-1)
    same = np.zeros(a.shape, dtype=bool)                            # one address: a broadcast
    same[..., 1:] = a[..., 1:] == a[..., :-1]
    slot = (a // 16) % 16
    cnt = ((slot[..., None] == np.arange(16)) & ~same[..., None]).sum(-2)
    return float(cnt.max(-1).mean())


def _pool_row_table(p: TilePlan, HH: int, HW: int) -> np.ndarray:
    """Row table of the fused-pool fp8 epilogue: every lane holds the 8 members of one 2^3
    window, one member per fragment (MT = 8), so the lane's running max over its fragments is
    the pooled value (the epilogue takes the window from any member's coordinates halved).
    Missing windows are dummy rows (-1).

    Bank slots: a ds_read_b128 lane group reads halo position hb at slot hb mod 16, and window
    bases are all even positions, so one member order for every lane puts a fragment's 16 rows
    on at most 8 slots (2.8 ways on the 128^3 conv4 plan, bank_ways).  Instead the windows are
    dealt to the 4 waves round-robin by base residue (so no slot is reachable from more than
    8 (lane, member) pairs of a wave), and each wave's bipartite multigraph lane -> slot (an
    edge per member, dummy lanes taking the slots' remaining degree) is 8-regular: it splits
    into 8 perfect matchings (Koenig), one per fragment -- 16 distinct slots in every fragment.
    Where the degrees do not allow it, the plain order (member m in fragment m) is kept."""
    assert p.MT == 8 and p.TD % 2 == 0 and p.TH % 2 == 0 and p.TW % 2 == 0
    wd, wh, ww = np.meshgrid(np.arange(p.TD // 2), np.arange(p.TH // 2), np.arange(p.TW // 2), indexing="ij")
    wd, wh, ww = wd.reshape(-1), wh.reshape(-1), ww.reshape(-1)
    nwin = wd.size
    assert nwin <= 64, "more windows than lanes x waves"
    md, mh, mw = np.arange(8) >> 2, (np.arange(8) >> 1) & 1, np.arange(8) & 1
    moff = (md * HH + mh) * HW + mw                              # halo offset of member m
    base = (2 * wd * HH + 2 * wh) * HW + 2 * ww

    def member_row(i, m):
        d, h, w = 2 * wd[i] + md[m], 2 * wh[i] + mh[m], 2 * ww[i] + mw[m]
        return ((d * HH + h) * HW + w, (d * p.TH + h) * p.TW + w)

    tab = np.zeros((4 * 8 * 16, 2), dtype=np.int32)
    tab[:, 1] = -1
    colored = _pool_coloring(base, moff, nwin)
    if colored is None:                           # plain order: window i -> wave i // 16, lane i % 16
        for i in range(nwin):
            wave, lr = divmod(i, 16)
            for m in range(8):
                tab[(wave * 8 + m) * 16 + lr] = member_row(i, m)
        return tab
    for wave, lanes, frag in colored:             # frag[f][lr] = (window, member) or (-1, slot)
        for f in range(8):
            for lr in range(16):
                i, m = frag[f][lr]
                tab[(wave * 8 + f) * 16 + lr] = member_row(i, m) if i >= 0 else (m, -1)
    return tab


def _pool_coloring(base: np.ndarray, moff: np.ndarray, nwin: int):
    """[(wave, windows, frag[8][16] of (window, member) | (-1, dummy slot))] or None (a slot
    reachable from more than 8 (lane, member) pairs of one wave)."""
    order = sorted(range(nwin), key=lambda i: (int(base[i]) % 16, i))
    waves = [order[w::4] for w in range(4)]
    out = []
    for wave, wins in enumerate(waves):
        if len(wins) > 16:
            return None
        # edges lane -> slot: (member list per (lane, slot)); lanes 0..len-1 are windows
        edges = [[[] for _ in range(16)] for _ in range(16)]
        deg = np.zeros(16, dtype=int)
        for lr, i in enumerate(wins):
            for m in range(8):
                r = int(base[i] + moff[m]) % 16
                edges[lr][r].append(m)
                deg[r] += 1
        if deg.max() > 8:
            return None
        spare = [r for r in range(16) for _ in range(8 - int(deg[r]))]   # 8 per dummy lane
        for k, lr in enumerate(range(len(wins), 16)):
            for r in spare[8 * k:8 * k + 8]:
                edges[lr][r].append(-1)
        frag = []
        for f in range(8):
            match_r = [-1] * 16                   # slot -> lane
            for lr in range(16):
                if not _augment(lr, edges, match_r, [False] * 16):
                    return None
            row = [None] * 16
            for r, lr in enumerate(match_r):
                m = edges[lr][r].pop()
                row[lr] = (wins[lr], m) if m >= 0 else (-1, r)
            frag.append(row)
        out.append((wave, wins, frag))
    return out


def _augment(lr, edges, match_r, seen) -> bool:
    """Kuhn's augmenting path from lane lr over slots with remaining edges."""
    for r in range(16):
        if edges[lr][r] and not seen[r]:
            seen[r] = True
            if match_r[r] < 0 or _augment(match_r[r], edges, match_r, seen):
                match_r[r] = lr
                return True
    return False


def natural_view(out_dims: tuple) -> tuple:
    """(osn, ob, osd, osh, osw) of a contiguous [N, OD, OH, OW, C] output."""
    OD, OH, OW = out_dims
    return (OD * OH * OW, 0, OH * OW, OW, 1)


def parity_view(full_dims: tuple, parity: tuple) -> tuple:
    """Output view writing position (d, h, w) of one parity class to (2d + jd, 2h + jh, 2w + jw)
    of a contiguous [N, FD, FH, FW, C] full-resolution output (sub-pixel upsample x2 convs)."""
    FD, FH, FW = full_dims
    jd, jh, jw = parity
    return (FD * FH * FW, (jd * FH + jh) * FW + jw, 2 * FH * FW, 2 * FW, 2)


def geometry(p: TilePlan, src_dims: tuple, out_dims: tuple, kdims: tuple, pads: tuple, view=None) -> list[int]:
    N, ID, IH, IW, C = src_dims
    OD, OH, OW = out_dims
    KD, KH, KW = kdims
    m = lambda v: int(np.int32(np.uint32(v)))    # noqa: E731 - unsigned magic as a signed int32
    return [N, ID, IH, IW, C, OD, OH, OW, KD, KH, KW, pads[0], pads[1], pads[2], p.TD, p.TH, p.TW,
            p.CS, p.HPpad, p.nks, p.nct, m(p.mHW), m(p.mHHW), p.BUF, m(_magic(p.TW)), m(_magic(p.TH))] + \
        list(view if view is not None else natural_view(out_dims))


def _dev_cached(cache: dict, device, make):
    key = str(device)
    t = cache.get(key)
    if t is None:
        t = make()
        with _LOCK:
            cache[key] = t
    return t


def zero_page(device) -> torch.Tensor:
    return _dev_cached(_ZERO, device, lambda: torch.zeros(64, dtype=torch.bfloat16, device=device))


def counters(cache: dict, lock, device, stream: int, n: int) -> torch.Tensor:
    """Zeroed int32 schedule counters, one buffer per (device, stream) -- kernels on one stream run
    in order and every launch leaves its counters zero.  Under hipGraph capture a stream's first
    use would record the zero fill into the graph (a fill kernel in every replay): the capture
    takes the device's eagerly made buffer instead (a captured step and eager launches on the same
    device do not run concurrently)."""
    key = (str(device), stream)
    t = cache.get(key)
    if t is None:
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            for (dev, _), u in list(cache.items()):
                if dev == str(device) and u.numel() == n:
                    return u
        t = torch.zeros(n, dtype=torch.int32, device=device)
        with lock:
            cache[key] = t
    return t


def sched(device, stream: int) -> torch.Tensor:
    # (conv_tile's dynamic schedules: a done counter + 8 XCD queue counters per column block)
    return counters(_SCHED, _LOCK, device, stream, 1024)


def rowtab_tensor(p: TilePlan, kdims: tuple, device) -> torch.Tensor:
    key = ("dev", p, tuple(kdims), str(device))
    t = _ROWTAB.get(key)
    if t is None:
        t = torch.from_numpy(row_table(p, kdims)).to(device)
        with _LOCK:
            _ROWTAB[key] = t
    return t


PD = 4                                           # B-ring depth of the kernel (k-steps in flight)
PD_F8 = 2                                        # (fp8 variant: 2 k-steps of 128)


def k_table(p: TilePlan, kdims: tuple) -> np.ndarray:
    """int32 [nks + 2 PD + 2, 4]: LDS byte offset of the tap that lane group lg (lanes 16lg ..
    16lg+15) reads in each k-step -- one tap for all four groups (CS >= 32: the groups take
    channel chunks of it), two taps (CS = 16: groups 0,1 / 2,3) or four (CS = 8); 0 past the
    last tap (zero weights).  fp8: four taps (CS = 32) or two (CS = 64, groups 0,1 / 2,3)."""
    KD, KH, KW = kdims
    HH, HW = p.TH + KH - 1, p.TW + KW - 1
    T = KD * KH * KW
    kd, kh, kw = np.meshgrid(np.arange(KD), np.arange(KH), np.arange(KW), indexing="ij")
    toff = (((kd * HH + kh) * HW + kw) * 16).reshape(-1)
    tab = np.zeros((p.nks + 2 * PD + 2, 4), dtype=np.int32)
    plane = p.HPpad * 16
    if p.f8 and p.bs:
        # block-scaled operand layout: row 2k = the tap offset of the scale lane group lg supplies
        # (32-k block lg of the MFMA), row 2k+1 = lg's packed data offsets lo | hi << 16 -- bytes 0-15
        # and 16-31 of its operand, two taps of one chunk plane (see conv_tile.hip read_a)
        tab2 = np.zeros((p.nks + 2 * PD + 2, 8), dtype=np.int64)
        off = lambda t: int(toff[t]) if t < T else 0   # noqa: E731
        for k in range(p.nks):
            for lg in range(4):
                if p.CS == 32:
                    st, lo, hi = 4 * k + lg, 4 * k + (lg >> 1), 4 * k + 2 + (lg >> 1)
                else:
                    st, lo, hi = 2 * k + (lg >> 1), 2 * k, 2 * k + 1
                assert off(lo) < 65536 and off(hi) < 65536
                tab2[k, lg] = off(st)
                tab2[k, 4 + lg] = off(lo) | (off(hi) << 16)
        return tab2.astype(np.uint32).view(np.int32).reshape(-1, 4)
    for k in range(p.nks):
        for lg in range(4):
            if p.f8:                                 # lane group: 32 bytes of one tap (planes in lb)
                t, off = (4 * k + lg, 0) if p.CS == 32 else (2 * k + lg // 2, 0)
            elif p.CS >= 32:
                t, s = divmod(k, p.CS // 32)
                off = s * 4 * plane
            elif p.CS == 16:
                t, off = 2 * k + lg // 2, 0
            else:
                t, off = 4 * k + lg, 0
            if t < T:
                tab[k, lg] = toff[t] + off
    return tab


def ktab_tensor(p: TilePlan, kdims: tuple, device) -> torch.Tensor:
    key = ("ktab", p, tuple(kdims), str(device))
    t = _ROWTAB.get(key)
    if t is None:
        t = torch.from_numpy(k_table(p, kdims)).to(device)
        with _LOCK:
            _ROWTAB[key] = t
    return t


def pack_weights(w: torch.Tensor, K: int, T: int, C: int, p: TilePlan, dgrad: bool) -> torch.Tensor:
    """Conv weight [K, taps, C] -> the kernel's fragment-ordered B stream (bf16), plus PD
    zero k-steps that the ring's over-the-end loads read (inside a ``packs.pack_scope``: from
    the model forward's one pack launch once recorded)."""
    desc = (K, T, C, p, bool(dgrad))
    hit = packs.lookup(w, desc, 5)
    if hit is not None:
        return hit
    Csrc = K if dgrad else C
    nslice = Csrc // p.CS
    out = torch.empty((nslice * p.nks + PD) * p.nct * 64 * 8, dtype=torch.bfloat16, device=w.device)
    wf = w.detach().float().contiguous()
    _native.kernels().tile_pack_w(wf.data_ptr(), out.data_ptr(), K, T, C, p.CS, p.nks, p.nct, nslice, int(dgrad),
                                  _native.stream(wf), p.NT)
    packs.record(w, desc, 5)
    return out


def _pack_job(w: torch.Tensor, desc, kind: int):
    """(job row, output, cache value) of one recorded tile-stream pack (packs.py kind 5)."""
    K, T, C, p, dgrad = desc
    nslice = (K if dgrad else C) // p.CS
    out = torch.empty((nslice * p.nks + PD) * p.nct * 64 * 8, dtype=torch.bfloat16, device=w.device)
    row = [w.data_ptr(), out.data_ptr(), 5, K, T, C, p.CS, p.nks, p.nct, nslice, int(dgrad), p.NT]
    return row, out, out


packs.register((5,), _pack_job, lambda desc, kind: desc[4])


def mask_dgrad_ok(p: TilePlan, ncol: int) -> bool:
    """The relu-mask dgrad epilogue fits: whole mask dwords per position and the two LDS mask
    buffers (rows x ncol / 8 bytes each, 256-B rounded) within the CU's LDS."""
    if ncol not in (32, 64):
        return False
    slots = 4 * p.MT * 16                        # (fragment-ordered mask slots)
    mb = -(-slots * (ncol // 8) // 256) * 256
    lds = 2 * p.BUF + 64 + red_bytes(p.NT) + (p.nks + 4 + 2) * 16 + p.HPpad * 8 + 2 * mb + 8 * slots
    return lds <= LDS_MAX


def _pack_params(p: TilePlan, Csrc: int, dgrad: bool) -> list[int]:
    return [p.CS, p.nks, p.nct, Csrc // p.CS, int(dgrad), p.NT]


def pack_pair(w: torch.Tensor, K: int, T: int, C: int, pf: TilePlan, pd: TilePlan):
    """(forward, dgrad) packed B streams of one weight in one launch (:func:`pack_weights`
    twice): the forward packs its backward's dgrad operand too (or both come from the scope's
    up-front launch)."""
    df, dd = (K, T, C, pf, False), (K, T, C, pd, True)
    hf, hd = packs.lookup(w, df, 5), packs.lookup(w, dd, 5)
    if hf is not None and hd is not None:
        return hf, hd
    outs = []
    for p, dg in ((pf, False), (pd, True)):
        Csrc = K if dg else C
        outs.append(torch.empty(((Csrc // p.CS) * p.nks + PD) * p.nct * 64 * 8, dtype=torch.bfloat16, device=w.device))
    wf = w.detach().float().contiguous()
    _native.kernels().tile_pack_w2(wf.data_ptr(), outs[0].data_ptr(), outs[1].data_ptr(), K, T, C,
                                   _pack_params(pf, C, False), _pack_params(pd, K, True), _native.stream(wf),
                                   [wf.numel(), outs[0].numel(), outs[1].numel()])
    packs.record(w, df, 5)
    packs.record(w, dd, 5)
    return outs[0], outs[1]


def workers(p: TilePlan, geom: list, ncol: int) -> int:
    """Rows of the BN-statistics slab a launch with statistics writes: one per chunk of tiles
    (conv_tile.hip's chunked deterministic schedule; the chunking depends on the tile count only)."""
    return int(_native.kernels().conv_tile_slab_rows(geom, ncol, p.NT))


def run(src5: torch.Tensor, wpk: torch.Tensor, bias, out: torch.Tensor, stats, p: TilePlan, geom: list, kdims: tuple,
        ncol: int, act: int, bny=None, bnp=None, oscale: float = 0.0, osc=None, pro=None) -> None:
    """``pro`` = (prm [4, C], act, z, mask or None): ``src5`` is a BN's pre-normalisation y and the
    kernel's loader applies z = act(y * prm[2] + prm[3]) to every landed halo, writing z (and the
    relu-mask bytes) for the positions its tiles own (conv_tile.hip ``xform_job``)."""
    st = _native.stream(src5)
    pk = {}
    if pro is not None:
        prm, pact, z, mask = pro
        assert prm.is_contiguous() and prm.shape == (4, src5.shape[-1]) and prm.dtype == torch.float32
        assert z is None or (z.is_contiguous() and z.numel() == src5.numel() and z.dtype == torch.bfloat16)
        pk = dict(pst=prm[2].data_ptr(), pz=_native.ptr(z), pmask=_native.ptr(mask), pact=int(pact),
                  pext=[2 * prm.shape[1], z.numel() if z is not None else 0, mask.numel() if mask is not None else 0])
    rt = rowtab_tensor(p, kdims, src5.device)
    kt = ktab_tensor(p, kdims, src5.device)
    ext = [src5.numel(), wpk.numel(), out.numel(), rt.numel() // 2, kt.numel() // 4]
    if bny is not None:
        ext += [bny.numel()] + ([bnp.numel()] if bnp is not None else [])
    _native.kernels().conv_tile(src5.data_ptr(), wpk.data_ptr(), rt.data_ptr(), kt.data_ptr(),
                                zero_page(src5.device).data_ptr(), _native.ptr(bias), out.data_ptr(),
                                _native.ptr(stats), geom, ncol, act, p.MT, p.NT, sched(src5.device, st).data_ptr(),
                                st, ext, _native.ptr(bny), _native.ptr(bnp), float(oscale), _native.ptr(osc),
                                osc.numel() if osc is not None else 0, **pk)


def conv_fwd(x5: torch.Tensor, w: torch.Tensor, bias, spec, act: int, want_stats: bool, p: TilePlan,
             out_scale: float | None = None, dstash: dict | None = None, pro=None):
    """y = act(conv(x, w) + b) (+ BN statistics slab) for a stride-1 conv on the tile kernel;
    ``out_scale``: e4m3 bytes of y / out_scale instead (fp8 inference input, no statistics).
    ``dstash`` (a dict kept by the caller until its backward): the dgrad's packed weights are made
    in the same launch and left there as ``(plan, packed)`` for :func:`conv_dgrad`.
    ``pro`` = (yb, prm, act, z, mask): x5 = z = act(bn(yb)) is not written yet -- the kernel reads
    yb, normalises in its loader and writes z (unless z is None: nothing will read it) and the mask
    (see :func:`run`)."""
    kd = (spec.KD, spec.KH, spec.KW)
    geom = geometry(p, (spec.N, spec.D, spec.H, spec.W, spec.C), (spec.OD, spec.OH, spec.OW), kd,
                    (spec.pd, spec.ph, spec.pw))
    pd = dgrad_plan(spec) if dstash is not None and not out_scale else None
    if pd is not None:
        wpk, wpk_d = pack_pair(w, spec.K, spec.taps, spec.C, p, pd)
        dstash["wpk"] = (pd, wpk_d)
    else:
        wpk = pack_weights(w, spec.K, spec.taps, spec.C, p, dgrad=False)
    y = torch.empty(spec.out_shape5, dtype=torch.uint8 if out_scale else torch.bfloat16, device=x5.device)
    stats = None
    if want_stats:
        assert not out_scale, "statistics with an fp8 output"
        stats = torch.empty(workers(p, geom, spec.K), 2, spec.K, dtype=torch.float32, device=x5.device)
    if pro is not None:
        assert not out_scale
        yb, prm, pact, z, mask = pro
        assert (z is None or z.data_ptr() == x5.data_ptr()) and yb.shape == x5.shape
        run(yb, wpk, bias, y, stats, p, geom, kd, spec.K, act, pro=(prm, pact, z, mask))
        return y, stats
    run(x5, wpk, bias, y, stats, p, geom, kd, spec.K, act, oscale=1.0 / out_scale if out_scale else 0.0)
    return y, stats


def conv_fwd_q8_block(x5: torch.Tensor, w: torch.Tensor, bias, spec, act: int, p: TilePlan):
    """The bf16 tile forward writing OCP MX-style block-scaled e4m3: (y bytes [N, OD, OH, OW, K],
    scales int32 [N, OD, OH, OW] -- byte j = E8M0 scale of channels 32j..32j+31).  The fp8 inference
    input of the next layer, from the epilogue (the space-to-depth stem instances)."""
    kd = (spec.KD, spec.KH, spec.KW)
    geom = geometry(p, (spec.N, spec.D, spec.H, spec.W, spec.C), (spec.OD, spec.OH, spec.OW), kd,
                    (spec.pd, spec.ph, spec.pw))
    wpk = pack_weights(w, spec.K, spec.taps, spec.C, p, dgrad=False)
    y = torch.empty(spec.out_shape5, dtype=torch.uint8, device=x5.device)
    ysc = torch.zeros(spec.out_shape5[:4], dtype=torch.int32, device=x5.device)
    run(x5, wpk, bias, y, None, p, geom, kd, spec.K, act, oscale=1.0, osc=ysc)
    return y, ysc


def conv_dgrad(dy5: torch.Tensor, w: torch.Tensor, spec, p: TilePlan, bn=None, wpk=None):
    """dx = conv(dy, flip(W)^T) with leading pads K-1-p (stride 1) on the tile kernel.

    ``bn = (y, prm, act)``: x was ``act(bn(y))`` with ``prm`` = (mean, invstd, scale, shift)
    [4, C]; the epilogue then also sums that BN's raw backward moments (sum g, sum g*y,
    g = dx * act'(z)) per workgroup and ``(dx, slab [workers, 2, C])`` is returned
    (``bn_finalize`` mode 2 turns them into dbeta, dgamma)."""
    kd = (spec.KD, spec.KH, spec.KW)
    geom = geometry(p, (spec.N, spec.OD, spec.OH, spec.OW, spec.K), (spec.D, spec.H, spec.W), kd,
                    (spec.KD - 1 - spec.pd, spec.KH - 1 - spec.ph, spec.KW - 1 - spec.pw))
    # ``wpk``: (plan, packed) left by the forward (:func:`conv_fwd` dstash), used when the plan matches
    wpk = wpk[1] if wpk is not None and wpk[0] == p else pack_weights(w, spec.K, spec.taps, spec.C, p, dgrad=True)
    dx = torch.empty(spec.N, spec.D, spec.H, spec.W, spec.C, dtype=torch.bfloat16, device=dy5.device)
    mask = bn[3] if bn is not None else None
    if bn is not None and mask is not None and mask_dgrad_ok(p, spec.C):
        # the relu-mask epilogue (statistics identity, ops/bnfuse.py): the slab's row 0 holds the
        # column sums of g = dx * relu'(z); dx itself is stored unmasked
        assert mask.numel() * 8 == dx.numel() and mask.dtype == torch.uint8
        slab = torch.empty(workers(p, geom, spec.C), 2, spec.C, dtype=torch.float32, device=dy5.device)
        run(dy5, wpk, None, dx, slab, p, geom, kd, spec.C, 0, bny=mask)
        return dx, ("identity", slab)
    run(dy5, wpk, None, dx, None, p, geom, kd, spec.C, 0)
    return dx if bn is None else (dx, None)


def fwd_plan(spec):
    if not enabled() or (spec.sd, spec.sh, spec.sw, spec.dd, spec.dh, spec.dw) != (1,) * 6:
        return None
    return plan(spec.N, (spec.OD, spec.OH, spec.OW), (spec.KD, spec.KH, spec.KW), spec.C, spec.K)


def dgrad_plan(spec):
    """dgrad into 64 columns (conv4's): 64-column workgroups -- one DMA of the 64-channel dy halo
    instead of one per 32-column block; that dgrad waited on its loader (profiles/r6_bn_prologue.md,
    waves addendum): 341.5 -> 312.5 us, where the 64-column forwards measured 1-2 % slower
    (profiles/r6_subpixel_nt4.md)."""
    if not enabled() or (spec.sd, spec.sh, spec.sw, spec.dd, spec.dh, spec.dw) != (1,) * 6:
        return None
    dims, kd = (spec.D, spec.H, spec.W), (spec.KD, spec.KH, spec.KW)
    return plan(spec.N, dims, kd, spec.K, spec.C, nt4=True) or plan(spec.N, dims, kd, spec.K, spec.C)


# ---------------------------------------------------------------------------
# kernel selection: the big-tile kernel vs conv_halo (deterministic, ops/tuning.py)
# ---------------------------------------------------------------------------
def choose(kind: str, spec, run_tile, run_other) -> bool:
    """True when the tile kernel should run ``kind`` ('fwd' / 'dgrad') of ``spec``.

    ``FN_CONV_TILE`` = 2 forces the tile kernel, 0 disables it; otherwise (default) the
    deterministic per-shape selection of :mod:`.tuning` decides (committed table, then the
    rule "tile whenever it plans"; ``FN_KERNEL_SELECT=autotune`` times unseen shapes)."""
    mode = os.environ.get("FN_CONV_TILE", "1")
    if mode == "0":
        return False
    if mode == "2":
        return True
    from . import tuning

    return tuning.select(kind, spec, run_tile, run_other)


# ---------------------------------------------------------------------------
# fp8 (e4m3) inference variant
# ---------------------------------------------------------------------------
def pack_weights_f8(wq: torch.Tensor, p: TilePlan) -> torch.Tensor:
    """e4m3 weight bytes [K, taps, C] (uint8) -> the fp8 kernel's fragment stream: uint8
    [(nslice * nks + 4) * nct * 64 * 32] -- per (slice, k-step, 16-column tile, lane) the 32
    bytes lane group lg multiplies (tap 4ks+lg x 32 channels for CS = 32, tap 2ks+lg/2 x
    channels 32(lg&1).. for CS = 64; block-scaled plans: bytes 0-15 / 16-31 of two taps, the
    halo's layout, see :func:`k_table`), columns in the bf16 kernel's permuted order, zeros past
    the last tap / column and 4 zero k-steps for the ring's over-the-end loads."""
    assert p.f8
    K, T, C = wq.shape
    nslice = C // p.CS
    tps = 128 // p.CS
    Tp = p.nks * tps
    wpad = torch.zeros(p.nct * 16, Tp, C, dtype=torch.uint8, device=wq.device)
    wpad[:K, :T] = wq
    sl, ks, ct, ln, i = np.meshgrid(np.arange(nslice), np.arange(p.nks), np.arange(p.nct), np.arange(64),
                                    np.arange(32), indexing="ij")
    fi, lg = ln & 15, ln >> 4
    col = (ct >> 1) * 32 + 8 * (fi >> 2) + 4 * (ct & 1) + (fi & 3)
    hi, b = i >> 4, i & 15
    if p.bs and p.CS == 32:
        tap, ch = 4 * ks + 2 * hi + (lg >> 1), sl * 32 + 16 * (lg & 1) + b
    elif p.bs:
        tap, ch = 2 * ks + hi, sl * 64 + 16 * lg + b
    elif p.CS == 32:
        tap, ch = 4 * ks + lg, sl * 32 + i
    else:
        tap, ch = 2 * ks + (lg >> 1), sl * 64 + 32 * (lg & 1) + i
    dev = wq.device
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a.reshape(-1))).to(dev)   # noqa: E731
    body = wpad[t(col), t(tap), t(ch)]
    return torch.cat([body, torch.zeros(4 * p.nct * 64 * 32, dtype=torch.uint8, device=dev)]).contiguous()


def conv_fwd_f8(xq5: torch.Tensor, wpk: torch.Tensor, scale: torch.Tensor, bias: torch.Tensor, spec, p: TilePlan,
                relu: bool, out_scale: float | None, i8: bool = False, xsc: torch.Tensor | None = None,
                out_block: bool = False):
    """y = act(conv(x, w) * scale + bias) of e4m3 activations (uint8 [N, D, H, W, C]) on the fp8
    tile kernel: bf16 output, or e4m3 of y / out_scale when ``out_scale`` is given.  ``i8``: the
    operands are int8 instead (x, wpk hold int8 bytes; the int8 MFMA instance).  A ``pool``
    plan returns maxpool2^3(relu(...)) instead: bf16 [N, OD/2, OH/2, OW/2, K].

    ``xsc`` (int32 [N, D, H, W]): block-scaled input -- byte j of a position's dword is the E8M0
    scale of its channels 32j..32j+31, applied by the scaled MFMA; ``scale`` then dequantises the
    weights only.  ``out_block`` (with xsc): block-scaled e4m3 output, returns ``(y, ysc)``."""
    kd = (spec.KD, spec.KH, spec.KW)
    geom = geometry(p, (spec.N, spec.D, spec.H, spec.W, spec.C), (spec.OD, spec.OH, spec.OW), kd,
                    (spec.pd, spec.ph, spec.pw))
    if p.pool:
        assert out_scale is None and relu
        y = torch.empty(spec.N, spec.OD // 2, spec.OH // 2, spec.OW // 2, spec.K, dtype=torch.bfloat16,
                        device=xq5.device)
    else:
        y = torch.empty(spec.out_shape5, dtype=torch.uint8 if (out_scale or out_block) else torch.bfloat16,
                        device=xq5.device)
    assert not out_block or (xsc is not None and not p.pool)
    ysc = torch.zeros(spec.out_shape5[:4], dtype=torch.int32, device=xq5.device) if out_block else None
    st = _native.stream(xq5)
    rt = rowtab_tensor(p, kd, xq5.device)
    kt = ktab_tensor(p, kd, xq5.device)
    oscale = 1.0 if out_block else (1.0 / out_scale if out_scale else 0.0)
    _native.kernels().conv_tile_f8(xq5.data_ptr(), wpk.data_ptr(), rt.data_ptr(), kt.data_ptr(),
                                   zero_page(xq5.device).data_ptr(), scale.data_ptr(), _native.ptr(bias), y.data_ptr(),
                                   oscale, geom, spec.K,
                                   int(relu) | (2 if p.pool else 0) | (4 if i8 else 0),
                                   p.MT, p.NT, st,
                                   sched(xq5.device, st).data_ptr(),
                                   [xq5.numel(), wpk.numel(), y.numel(), rt.numel() // 2, kt.numel() // 4,
                                    xsc.numel() if xsc is not None else 0, ysc.numel() if ysc is not None else 0],
                                   _native.ptr(xsc), _native.ptr(ysc))
    return (y, ysc) if out_block else y
