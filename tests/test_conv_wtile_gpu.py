"""Big-tile weight-gradient kernel (``csrc/kernels/conv_wtile.hip``) vs the fp32 reference.

FeatureNet-3D layer shapes at a small batch and at production-size batches whose tile
count is many times the workgroups of every (XCD, column group) (static per-workgroup tile
sets, double-buffered jobs), the segmentation decoder conv ('same' padding, 64 input
channels = 4 slices), a 2-D conv, Cout 16, in-place accumulation into ``out`` and
repeated launches (accumulating into the same output).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

from featurenet_amd import _native  # noqa: E402
from featurenet_amd.ops import conv_wtile as cw  # noqa: E402
from featurenet_amd.ops import reference as ref  # noqa: E402
from featurenet_amd.ops.spec import ConvSpec  # noqa: E402


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item(), (a - b).abs().max().item() / (b.abs().max().item() + 1e-12)


CASES = [
    # (N, D, H, W, C, K, kernel, padding)
    (2, 29, 29, 29, 32, 32, (5, 5, 5), "valid"),     # FeatureNet-3D conv2 (2 tap groups x 2 slices)
    (2, 25, 25, 25, 32, 64, (4, 4, 4), "valid"),     # conv3
    (2, 22, 22, 22, 64, 64, (3, 3, 3), "valid"),     # conv4 (4 slices, dead taps 27..31)
    (24, 29, 29, 29, 32, 32, (5, 5, 5), "valid"),    # conv2 at a production batch: many jobs per workgroup
    (32, 22, 22, 22, 64, 64, (3, 3, 3), "valid"),    # conv4 at a production batch
    (3, 24, 24, 24, 64, 32, (3, 3, 3), "same"),      # segmentation decoder conv (padding, edge tiles)
    (4, 1, 40, 37, 32, 32, (1, 5, 5), "same"),       # 2-D conv
    (2, 14, 15, 16, 16, 16, (3, 3, 3), "same"),      # Cout 16
    # 8 input channels (two taps per B fragment): the space-to-depth stem of FeatureNet-3D
    # (7^3 stride 2 on 64^3 -> 4^3 stride 1 on 8 channels of a 32^3 grid)
    (2, 32, 32, 32, 8, 32, (4, 4, 4), "valid"),
    (24, 32, 32, 32, 8, 32, (4, 4, 4), "valid"),     # at a production batch
    (3, 20, 21, 22, 8, 64, (3, 3, 3), "same"),       # odd kernel (tap pairs straddle kw rows), edges
]


def _case(case, seed=0):
    N, D, H, W, C, K, k, pad = case
    torch.manual_seed(seed)
    x = torch.randn(N, D, H, W, C, device="cuda").to(torch.bfloat16)
    spec = ConvSpec.make(x.shape, K, k, 1, pad)
    dy = torch.randn(spec.out_shape5, device="cuda").to(torch.bfloat16)
    return x, dy, spec


def _ref_dw(x, dy, spec):
    w = torch.zeros(spec.K, spec.KD, spec.KH, spec.KW, spec.C, device="cuda", requires_grad=True)
    y = ref.conv(x.float(), w, None, spec)
    y.backward(dy.float())
    return w.grad


@pytest.mark.parametrize("case", CASES)
def test_wtile_wgrad_matches_reference(case):
    assert _native.kernels_available()
    x, dy, spec = _case(case)
    p = cw.plan(spec)
    assert p is not None, spec
    dw = cw.conv_wgrad(dy, x, spec, p)
    rel, mx = _rel(dw, _ref_dw(x, dy, spec))
    assert rel < 5e-3 and mx < 2e-2, (case, p, rel, mx)


def test_wtile_accumulates_into_out_and_repeats():
    x, dy, spec = _case(CASES[0], seed=3)
    p = cw.plan(spec)
    want = _ref_dw(x, dy, spec)
    out = torch.zeros(spec.K, spec.taps, spec.C, dtype=torch.float32, device="cuda")
    for _ in range(3):                               # three launches accumulate 3x
        cw.conv_wgrad(dy, x, spec, p, out=out)
    rel, mx = _rel(out.reshape(want.shape) / 3, want)
    assert rel < 5e-3 and mx < 2e-2, (rel, mx)


@pytest.mark.parametrize("case", [CASES[2], CASES[4], CASES[5], CASES[6], CASES[8], CASES[9]])
def test_wtile_kstep_split_matches_unsplit(case, monkeypatch):
    """The k-step split (two partial slabs per worker) against the fp32 oracle, with the
    unsplit plan of the same shape as a second opinion."""
    x, dy, spec = _case(case, seed=5)
    want = _ref_dw(x, dy, spec)
    got = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("FN_WTILE_KS2", flag)
        cw._PLANS.clear()
        p = cw.plan(spec)
        assert p is not None and p.ks2 == (flag == "1"), (case, p)
        got[flag] = cw.conv_wgrad(dy, x, spec, p)
        rel, mx = _rel(got[flag], want)
        assert rel < 5e-3 and mx < 2e-2, (case, p, rel, mx)
    cw._PLANS.clear()
    rel, _ = _rel(got["1"], got["0"])
    assert rel < 2e-3
