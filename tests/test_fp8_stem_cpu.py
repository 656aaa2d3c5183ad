"""The fp8 stem's tap-expanded space-to-depth formulation (``inference/fp8.py``) is the
same convolution: a 7^3 stride-2 'valid' conv over 1 channel == a (4, 4, 1)-tap conv over
the 32-channel packed input with the folded weight (fp32, CPU; the packing is emulated
in torch with the ``s2d_tap_f8`` kernel's index map)."""
import torch
import torch.nn.functional as F

from featurenet_amd.inference.fp8 import stem_tap_plan, stem_tap_weight


class _Stem:
    kernel, stride, padding, cout = (7, 7, 7), (2, 2, 2), "valid", 8


def _tap_input(x, spec):
    """y[n, d, h, w, 8j + pd*4 + ph*2 + pw] = x[n, 2d+pd, 2h+ph, 2(w+j)+pw] (0 outside)."""
    N, D, H, W, _ = x.shape
    y = torch.zeros(N, spec.D, spec.H, spec.W, 32)
    for j in range(4):
        for pd in range(2):
            for ph in range(2):
                for pw in range(2):
                    for d in range(spec.D):
                        for h in range(spec.H):
                            xd, xh = 2 * d + pd, 2 * h + ph
                            if xd >= D or xh >= H:
                                continue
                            xw = 2 * (torch.arange(spec.W) + j) + pw
                            ok = xw < W
                            y[:, d, h, ok, 8 * j + pd * 4 + ph * 2 + pw] = x[:, xd, xh, xw[ok], 0]
    return y


def test_stem_tap_expansion_is_the_strided_conv():
    torch.manual_seed(0)
    x = torch.randn(2, 24, 22, 26, 1)
    w = torch.randn(8, 7, 7, 7, 1)
    spec = stem_tap_plan(_Stem, tuple(x.shape))
    assert spec is not None and spec.C == 32 and (spec.KD, spec.KH, spec.KW) == (4, 4, 1)
    ref = F.conv3d(x.permute(0, 4, 1, 2, 3), w.permute(0, 4, 1, 2, 3), stride=2).permute(0, 2, 3, 4, 1)
    xt = _tap_input(x, spec)
    wt = stem_tap_weight(w)
    got = F.conv3d(xt.permute(0, 4, 1, 2, 3), wt.permute(0, 4, 1, 2, 3)).permute(0, 2, 3, 4, 1)
    assert got.shape == ref.shape
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)


def test_stem_tap_plan_rejects_other_stems():
    class S(_Stem):
        kernel = (5, 5, 5)
    assert stem_tap_plan(S, (1, 32, 32, 32, 1)) is None            # ceil(5/2) = 3 taps
    assert stem_tap_plan(_Stem, (1, 32, 32, 32, 2)) is None         # 2 input channels
