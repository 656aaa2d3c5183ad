"""Host planning of the big-tile weight-gradient kernel (``ops/conv_wtile.py``), CPU only.

The row table must cover every output position of a tile exactly once and order the
k-rows so a transposed LDS read of 8 rows touches 64 distinct banks; the 8-channel
(stem) form reads 16-B positions at hpos and hpos + 1, so each group of 8 rows takes 8
distinct residues mod 16 of one parity.
"""
import numpy as np
import pytest

from featurenet_amd.ops import conv_wtile as cw
from featurenet_amd.ops.spec import ConvSpec


def _plan(case, nw="8", monkeypatch=None):
    N, D, H, W, C, K, k, pad = case
    if monkeypatch is not None:
        monkeypatch.setenv("FN_WTILE_NW", nw)
    cw._PLANS.clear()
    spec = ConvSpec.make((N, D, H, W, C), K, k, 1, pad)
    return spec, cw.plan(spec)


@pytest.mark.parametrize("case", [
    (128, 32, 32, 32, 8, 32, (4, 4, 4), "valid"),    # FeatureNet-3D stem after space-to-depth
    (128, 29, 29, 29, 32, 32, (5, 5, 5), "valid"),   # conv2
    (128, 22, 22, 22, 64, 64, (3, 3, 3), "valid"),   # conv4
])
def test_row_table_covers_tile_and_spreads_banks(case, monkeypatch):
    spec, p = _plan(case, "8", monkeypatch)
    assert p is not None and p.nw == 8
    assert p.c8 == (spec.C == 8)
    rows, pos = cw.tables(p, (spec.KD, spec.KH, spec.KW))
    assert rows.shape == (p.kst * 32, 2) and pos.shape == (p.HPpad,)
    real = rows[rows[:, 1] >= 0]
    assert len(real) == p.rows and len(set(real[:, 1].tolist())) == p.rows
    h = rows[:, 0] // p.xr
    assert (h >= 0).all() and (h < p.HPpad).all() and (pos[h] >= 0).all()
    bad = 0
    for g in range(len(h) // 8):
        hs = h[8 * g: 8 * g + 8]
        if p.c8:
            banks = {x % 16 for x in hs} | {(x + 1) % 16 for x in hs}
            bad += len(banks) < 16
        else:
            bad += len({x % 8 for x in hs}) < 8
    assert bad <= max(1, len(h) // 8 // 10), (bad, len(h) // 8)    # overflow rows only


def test_stem_geometry_is_launchable(monkeypatch):
    spec, p = _plan((128, 32, 32, 32, 8, 32, (4, 4, 4), "valid"), "8", monkeypatch)
    g = cw.geometry(p, spec)
    assert g[20] == p.HPpad * 16 and p.HPpad % 64 == 0       # XB: whole 64-position DMA instructions
    assert p.BUF >= g[20] + p.kst * 32 * spec.K * 2 and p.BUF % 1024 == 0
    assert p.ntg == 1 and p.G == 1                           # 4 waves x 8 fragments x 2 taps = 64 taps
    assert p.ks2 and cw.flags(p) == 8 | (8 << 8) | (1 << 12) | (1 << 13)
    lds = 2 * p.BUF + 64 + p.kst * 32 * 12 + p.HPpad * 8
    assert lds <= cw.LDS_MAX


def test_four_wave_mode_keeps_sixteen_channel_rule(monkeypatch):
    spec, p = _plan((128, 32, 32, 32, 8, 32, (4, 4, 4), "valid"), "4", monkeypatch)
    assert p is None                                          # the loader variant needs C % 16 == 0
    cw._PLANS.clear()


@pytest.mark.parametrize("case,ks2", [
    ((128, 32, 32, 32, 8, 32, (4, 4, 4), "valid"), True),      # stem: 4 fragments of 2 taps -> 8
    ((128, 22, 22, 22, 64, 64, (3, 3, 3), "valid"), True),     # conv4: T = 27 <= 32
    ((128, 64, 64, 64, 64, 32, (3, 3, 3), "same"), True),      # seg decoder conv
    ((128, 29, 29, 29, 32, 32, (5, 5, 5), "valid"), False),    # conv2: 16 fragments already
    ((128, 25, 25, 25, 32, 64, (4, 4, 4), "valid"), False),    # conv3: 8 fragments of Cout 64
])
def test_kstep_split_selection(case, ks2, monkeypatch):
    spec, p = _plan(case, "8", monkeypatch)
    assert p.ks2 == ks2 and p.kst >= 2
    wpt = 4 if p.ks2 else 8
    assert p.ntg == -(-spec.taps // (wpt * p.nacc * (2 if p.c8 else 1)))
    monkeypatch.setenv("FN_WTILE_KS2", "0")
    cw._PLANS.clear()
    assert not cw.plan(spec).ks2
    cw._PLANS.clear()
