"""Sub-pixel decomposition of upsample x2 + 3^3 'same' conv (ops/subpixel.py), CPU fp64.

Forward through the 8 parity classes, dgrad as one 2^3 conv over the shifted
space-to-depth view of dy, and the weight gradient as the adjoint weight fold of the
per-class gradients -- each against autograd through the materialised upsample.
"""
import torch
import torch.nn.functional as F

from featurenet_amd.ops import subpixel as sp


def _direct(x, w):
    up = x.repeat_interleave(2, 1).repeat_interleave(2, 2).repeat_interleave(2, 3)
    y = F.conv3d(up.permute(0, 4, 1, 2, 3), w.permute(0, 4, 1, 2, 3), padding=1)
    return y.permute(0, 2, 3, 4, 1)


def _data(seed=0, N=2, D=3, H=4, W=5, C=3, K=2):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, D, H, W, C, generator=g, dtype=torch.float64)
    w = torch.randn(K, 3, 3, 3, C, generator=g, dtype=torch.float64)
    dy = torch.randn(N, 2 * D, 2 * H, 2 * W, K, generator=g, dtype=torch.float64)
    return x, w, dy


def test_forward_classes_match_upsample_conv():
    x, w, _ = _data()
    torch.testing.assert_close(sp.ref_forward(x, w), _direct(x, w))


def test_shift_roundtrip_and_border():
    _, _, dy = _data(1)
    sh = sp.shift_s2d(dy)
    assert sh.shape == (2, 4, 5, 6, 16)
    torch.testing.assert_close(sp.unshift_s2d(sh, 2), dy)
    # cell 0 sub-position 0 along D is the full-res position -1: zero
    assert sh[:, 0].reshape(2, 5, 6, 2, 2, 2, 2)[:, :, :, 0].abs().max() == 0


def test_dgrad_is_conv_over_shifted_view():
    x, w, dy = _data(2)
    x.requires_grad_(True)
    (_direct(x, w) * dy).sum().backward()
    torch.testing.assert_close(sp.ref_dgrad(dy, w), x.grad)


def test_weight_grad_is_adjoint_fold():
    x, w, dy = _data(3)
    w.requires_grad_(True)
    (_direct(x, w) * dy).sum().backward()
    dwf = sp.ref_wgrad_classes(dy, x)
    torch.testing.assert_close(sp.fold_weight_grad(dwf), w.grad)


def test_fold_is_adjoint_of_forward_weights():
    g = torch.Generator().manual_seed(4)
    w = torch.randn(3, 3, 3, 3, 5, generator=g, dtype=torch.float64)
    v = torch.randn(8, 3, 2, 2, 2, 5, generator=g, dtype=torch.float64)
    lhs = (sp.forward_weights(w) * v).sum()
    rhs = (w * sp.fold_weight_grad(v)).sum()
    torch.testing.assert_close(lhs, rhs)
