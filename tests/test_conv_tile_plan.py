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
    assert p.BUF >= p.HPpad * (p.CS // 8) * 16
    assert 2 * p.BUF + 64 + ct.RED_BYTES + (p.nks + ct.PD + 2) * 8 + p.HPpad * 8 <= ct.LDS_MAX
    HP = (p.TD + k[0] - 1) * (p.TH + k[1] - 1) * (p.TW + k[2] - 1)
    assert p.HPpad >= HP and p.HPpad % 64 == 0
    tab = ct.row_table(p, k)
    assert tab.shape == (4 * p.MT * 16, 2)
    nat = tab[:, 1][tab[:, 1] >= 0]
    assert sorted(nat.tolist()) == list(range(p.rows))          # every tile row exactly once
    HH, HW = p.TH + k[1] - 1, p.TW + k[2] - 1
    toff_max = ((k[0] - 1) * HH + k[1] - 1) * HW + k[2] - 1
    assert tab[:, 0].max() + toff_max < HP                        # every A read inside the halo


@pytest.mark.parametrize("out,k,c,n", FEATURENET)
def test_featurenet_fragments_nearly_conflict_free(out, k, c, n):
    """The planner may trade a few repeated bank slots for a smaller halo (its cost model
    charges them); at most 10% of the fragment slots of a FeatureNet layer repeat."""
    p = ct.plan(128, out, k, c, n)
    res = ct.row_table(p, k)[:, 0].reshape(-1, 16) % 16
    dups = sum(16 - len(set(r.tolist())) for r in res)
    assert dups <= 0.1 * res.size


def test_row_table_conflict_free_when_residues_allow():
    # 5x5x20 tile of a 3^3 conv: 7x7x22 halo, every residue class has >= 32 rows
    p = ct.TilePlan(5, 5, 20, 32, 8, 2, 1088, 28, 4, 1088 * 64, ct._magic(22), ct._magic(7 * 22), 0.0)
    res = ct.row_table(p, (3, 3, 3))[:, 0].reshape(-1, 16) % 16
    assert all(len(set(r.tolist())) == 16 for r in res)


def test_magic_division_exact():
    for HH, HW in [(9, 29), (14, 25), (7, 22), (13, 28), (15, 33)]:
        assert ct._magic_ok(HH, HW, 4096)
