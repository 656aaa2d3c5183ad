"""Planner and row-table logic of the big-tile conv kernel (CPU only)."""
import numpy as np
import pytest

from featurenet_amd.ops import conv_tile as ct

FEATURENET = [((25, 25, 25), (5, 5, 5), 32, 32), ((22, 22, 22), (4, 4, 4), 32, 64),
              ((20, 20, 20), (3, 3, 3), 64, 64), ((29, 29, 29), (5, 5, 5), 32, 32),
              ((25, 25, 25), (4, 4, 4), 64, 32), ((22, 22, 22), (3, 3, 3), 64, 64)]


@pytest.mark.parametrize("out,k,c,n", FEATURENET)
def test_plans_fit_lds_and_cover_rows(out, k, c, n):
    p = ct.plan(128, out, k, c, n)
    assert p is not None
    assert 2 * p.BUF + 64 + 1024 + 4 * 64 * p.MT * 4 <= ct.LDS_MAX
    HP = (p.TD + k[0] - 1) * (p.TH + k[1] - 1) * (p.TW + k[2] - 1)
    assert p.HPpad >= HP and p.HPpad % 64 == 0
    tab = ct.row_table(p, k)
    assert tab.shape == (4 * p.MT * 16, 2)
    nat = tab[:, 1][tab[:, 1] >= 0]
    assert sorted(nat.tolist()) == list(range(p.rows))          # every tile row exactly once
    HH, HW = p.TH + k[1] - 1, p.TW + k[2] - 1
    toff_max = ((k[0] - 1) * HH + k[1] - 1) * HW + k[2] - 1
    assert tab[:, 0].max() + toff_max < HP                        # every A read inside the halo


@pytest.mark.parametrize("out,k,c,n", [f for f in FEATURENET if f[0] != (25, 25, 25) or f[2] != 64])
def test_featurenet_fragments_conflict_free(out, k, c, n):
    p = ct.plan(128, out, k, c, n)
    res = ct.row_table(p, k)[:, 0].reshape(-1, 16) % 16
    assert all(len(set(r.tolist())) == 16 for r in res)


def test_magic_division_exact():
    for HH, HW in [(9, 29), (14, 25), (7, 22), (13, 28), (15, 33)]:
        assert ct._magic_ok(HH, HW, 4096)
