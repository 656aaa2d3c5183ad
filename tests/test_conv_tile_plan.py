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
    assert 2 * p.BUF + 64 + ct.red_bytes(p.NT) + (p.nks + ct.PD + 2) * 16 + p.HPpad * 8 + 256 <= ct.LDS_MAX
    assert p.NT == 2
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


def test_bank_ways_matches_row_residues():
    """bank_ways: 1.0 for a fragment set with 16 distinct residues and one tap per lane group
    pair (CS = 32); a plan whose fragments repeat residues reads more than 1-way; CS = 8 (four
    taps per k-step, the ds_read_b128 groups mixing two lane groups) shifts residues."""
    p = ct.TilePlan(5, 5, 20, 32, 8, 2, 1088, 28, 4, 1088 * 64, ct._magic(22), ct._magic(7 * 22), 0.0)
    assert ct.bank_ways(p, (3, 3, 3)) == 1.0
    q = ct.plan(128, (20, 20, 20), (3, 3, 3), 64, 64)           # conv4 fwd: 5x10x10, 44 repeated slots
    res = ct.row_table(q, (3, 3, 3))[:, 0].reshape(-1, 16) % 16
    if any(len(set(r.tolist())) < 16 for r in res):
        assert ct.bank_ways(q, (3, 3, 3)) > 1.0
    s = ct.plan(128, (29, 29, 29), (4, 4, 4), 8, 32)             # the stem (CS = 8)
    assert 1.0 <= ct.bank_ways(s, (4, 4, 4)) <= 4.0


def test_magic_division_exact():
    for HH, HW in [(9, 29), (14, 25), (7, 22), (13, 28), (15, 33)]:
        assert ct._magic_ok(HH, HW, 4096)


@pytest.mark.parametrize("out,k,c,n", [((57, 57, 57), (5, 5, 5), 32, 32), ((54, 54, 54), (4, 4, 4), 32, 64),
                                       ((52, 52, 52), (3, 3, 3), 64, 64)])
def test_fp8_plans_and_weight_stream(out, k, c, n):
    """fp8 tile plans (128^3 inference layers): 32-/64-channel slices, 128-k steps in ring-depth
    pairs, and the packed e4m3 stream holds w[col][tap][ch] where the kernel's lane map says."""
    import torch
    p = ct.plan(128, out, k, c, n, f8=True)
    assert p is not None and p.f8 and p.CS in (32, 64) and p.MT == 8
    T = k[0] * k[1] * k[2]
    tps = 128 // p.CS
    assert p.nks % ct.PD_F8 == 0 and p.nks * tps >= T
    assert 2 * p.BUF + 64 + ct.red_bytes(p.NT, True) + (p.nks + ct.PD_F8 + 2) * 16 + p.HPpad * 8 <= ct.LDS_MAX
    g = torch.Generator().manual_seed(0)
    wq = torch.randint(1, 255, (n, T, c), generator=g, dtype=torch.uint8)
    wpk = ct.pack_weights_f8(wq, p)
    nslice = c // p.CS
    assert wpk.numel() == (nslice * p.nks + 4) * p.nct * 64 * 32
    frag = wpk.reshape(-1, p.nct, 64, 32)
    assert not frag[nslice * p.nks:].any()                       # the ring's zero k-steps
    for sl, ks, cti, lane in [(0, 0, 0, 0), (nslice - 1, p.nks - 1, p.nct - 1, 63), (0, 1, 1, 37)]:
        fi, lg = lane & 15, lane >> 4
        col = (cti >> 1) * 32 + 8 * (fi >> 2) + 4 * (cti & 1) + (fi & 3)
        tap = 4 * ks + lg if p.CS == 32 else 2 * ks + (lg >> 1)
        ch0 = sl * p.CS + (0 if p.CS == 32 else 32 * (lg & 1))
        want = wq[col, tap, ch0:ch0 + 32] if (tap < T and col < n) else torch.zeros(32, dtype=torch.uint8)
        assert torch.equal(frag[sl * p.nks + ks, cti, lane], want)
    kt = ct.k_table(p, k)
    HH, HW = p.TH + k[1] - 1, p.TW + k[2] - 1
    t = min(5, T - 1)
    kd, r = divmod(t, k[1] * k[2])
    kh, kw = divmod(r, k[2])
    ks, lg = (t // 4, t % 4) if p.CS == 32 else (t // 2, 2 * (t % 2))
    assert kt[ks, lg] == ((kd * HH + kh) * HW + kw) * 16


@pytest.mark.parametrize("out,k,c,n", [((52, 52, 52), (3, 3, 3), 64, 64), ((20, 20, 20), (3, 3, 3), 64, 64),
                                       ((10, 12, 14), (3, 3, 3), 32, 32)])
def test_fp8_pool_plans_hold_whole_windows_per_lane(out, k, c, n):
    """Fused-pool fp8 plans: even tile dims, and lane lr of wave w holds the 8 members of one
    2^3 window in fragments 0..7 (each tile row exactly once, any member order); the
    edge-coloured table reads conflict-free (16 distinct slots per fragment)."""
    p = ct.plan(64, out, k, c, n, f8=True, pool=True)
    assert p is not None and p.pool and p.MT == 8
    assert p.TD % 2 == 0 and p.TH % 2 == 0 and p.TW % 2 == 0
    tab = ct.row_table(p, k)
    nat = tab[:, 1][tab[:, 1] >= 0]
    assert sorted(nat.tolist()) == list(range(p.rows))
    t = tab[:, 1].reshape(4, 8, 16)                  # [wave][fragment][lane]
    for wv in range(4):
        for lr in range(16):
            rows = t[wv, :, lr]
            if rows[0] < 0:
                assert (rows < 0).all()
                continue
            tw, th, td = rows % p.TW, (rows // p.TW) % p.TH, rows // (p.TW * p.TH)
            assert len({(a // 2, b // 2, e // 2) for a, b, e in zip(td, th, tw)}) == 1   # one window
            assert len({(a % 2, b % 2, e % 2) for a, b, e in zip(td, th, tw)}) == 8      # 8 members
    if p.CS == 64:
        assert ct.bank_ways(p, k) == 1.0
    assert ct.plan(64, (21, 20, 20), k, c, n, f8=True, pool=True) is None           # odd output dim
