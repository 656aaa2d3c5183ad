"""CPU oracle semantics: Keras 'same' padding, pooling, BN, loss, flat optimizers.

The HIP kernels are checked against these oracles in ``test_kernels_gpu.py``;
here the oracles themselves are pinned against naive loop implementations of
the Keras/TF semantics the reference relies on (asymmetric 'same' padding with
the extra pad on the high side, pooling windows that ignore padding).
"""
import itertools

import numpy as np
import pytest
import torch

from featurenet_amd.ops import reference as R
from featurenet_amd.ops.spec import ConvSpec, PoolSpec, same_pad


def _naive_conv(x, w, b, spec):
    N, D, H, W, C = x.shape
    K = w.shape[0]
    out = np.zeros((N, spec.OD, spec.OH, spec.OW, K), np.float64)
    for n, od, oh, ow in itertools.product(range(N), range(spec.OD), range(spec.OH), range(spec.OW)):
        acc = np.zeros(K)
        for kd, kh, kw in itertools.product(range(spec.KD), range(spec.KH), range(spec.KW)):
            d = od * spec.sd - spec.pd + kd * spec.dd
            h = oh * spec.sh - spec.ph + kh * spec.dh
            ww = ow * spec.sw - spec.pw + kw * spec.dw
            if 0 <= d < D and 0 <= h < H and 0 <= ww < W:
                acc += w[:, kd, kh, kw, :] @ x[n, d, h, ww, :]
        out[n, od, oh, ow] = acc + (b if b is not None else 0)
    return out


def test_same_pad_matches_tf():
    # TF: out = ceil(in/s); total = max((out-1)*s + k - in, 0); lo = total//2
    assert same_pad(5, 2, 2) == (0, 1)
    assert same_pad(64, 7, 2) == (2, 3)
    assert same_pad(7, 3, 1) == (1, 1)
    assert same_pad(4, 1, 2) == (0, 0)


@pytest.mark.parametrize("shape,k,s,pad", [((1, 5, 6, 7, 3), (3, 2, 3), (2, 1, 2), "same"),
                                           ((2, 6, 6, 6, 2), (3, 3, 3), (1, 1, 1), "valid"),
                                           ((1, 1, 9, 9, 4), (1, 5, 5), (1, 2, 2), "same")])
def test_conv_oracle_vs_naive(shape, k, s, pad):
    rng = np.random.default_rng(0)
    x = rng.standard_normal(shape)
    spec = ConvSpec.make(shape, 5, k, s, pad)
    w = rng.standard_normal((5,) + tuple(k) + (shape[-1],))
    b = rng.standard_normal(5)
    got = R.conv(torch.tensor(x), torch.tensor(w), torch.tensor(b), spec).numpy()
    np.testing.assert_allclose(got, _naive_conv(x, w, b, spec), rtol=1e-9, atol=1e-9)


def test_maxpool_same_ignores_padding():
    x = -torch.ones(1, 1, 5, 5, 1, dtype=torch.float64)
    spec = PoolSpec.make(x.shape, (1, 2, 2), (1, 2, 2), "same")
    y = R.pool(x, spec, "max")
    assert y.shape == (1, 1, 3, 3, 1)
    assert torch.all(y == -1)                         # -inf padding never wins
    ya = R.pool(torch.ones_like(x), spec, "avg")
    assert torch.allclose(ya, torch.ones_like(ya))    # Keras avg excludes padding


def test_batchnorm_act_oracle():
    torch.manual_seed(0)
    y = torch.randn(4, 3, 3, 3, 6, dtype=torch.float64)
    g, b = torch.rand(6, dtype=torch.float64) + 0.5, torch.randn(6, dtype=torch.float64)
    rm, rv = torch.zeros(6, dtype=torch.float64), torch.ones(6, dtype=torch.float64)
    z = R.batchnorm_act(y, g, b, rm, rv, True, 0.01, 1e-3, "relu")
    flat = y.reshape(-1, 6)
    mu, var = flat.mean(0), flat.var(0, unbiased=False)
    ref = torch.relu((flat - mu) / torch.sqrt(var + 1e-3) * g + b).reshape(y.shape)
    torch.testing.assert_close(z, ref)
    n = flat.shape[0]
    torch.testing.assert_close(rm, 0.01 * mu)
    torch.testing.assert_close(rv, 0.99 + 0.01 * flat.var(0, unbiased=True))
    assert n == 108


def test_softmax_xent_smoothing():
    logits = torch.tensor([[2.0, 0.0, -1.0]])
    y = torch.tensor([0])
    p = torch.softmax(logits, -1)
    ref = -(0.9 * torch.log(p[0, 0]) + 0.1 / 3 * torch.log(p[0]).sum())
    torch.testing.assert_close(R.softmax_xent(logits, y, 0.1), ref)


def test_flat_adam_matches_keras_formula():
    from featurenet_amd.ops.optim import FlatAdam

    p = torch.tensor([1.0, -2.0, 3.0])
    g = torch.tensor([0.1, 0.2, -0.3])
    opt = FlatAdam(p, g, lr=0.01, keras_eps=True)
    p0 = p.clone()
    opt.step()
    # Keras 2 Adam: lr_t = lr*sqrt(1-b2)/(1-b1); p -= lr_t*m/(sqrt(v)+eps)
    m, v = 0.1 * g, 0.001 * g * g
    lr_t = 0.01 * np.sqrt(1 - 0.999) / (1 - 0.9)
    torch.testing.assert_close(p, p0 - lr_t * m / (torch.sqrt(v) + opt.eps), rtol=1e-5, atol=1e-7)


def test_flat_sgd_momentum():
    from featurenet_amd.ops.optim import FlatSGD

    p = torch.tensor([1.0])
    g = torch.tensor([0.5])
    opt = FlatSGD(p, g, lr=0.1, momentum=0.9)
    opt.step()
    opt.step()
    # v1 = -0.05 ; p1 = 0.95 ; v2 = 0.9*-0.05 - 0.05 = -0.095 ; p2 = 0.855
    torch.testing.assert_close(p, torch.tensor([0.855]))


def test_eval_bn_folding_matches_unfolded_bn():
    """Eval-mode Conv folds BN into the conv weights/bias; same result as conv -> BN(running) -> act -> pool."""
    from featurenet_amd.models.layers import Conv
    from featurenet_amd.ops import reference as R

    torch.manual_seed(0)
    m = Conv(4, 8, 3, 1, "same", bn=True, act="relu", pool=2)
    with torch.no_grad():
        m.gamma.uniform_(0.5, 1.5)
        m.beta.uniform_(-0.3, 0.3)
        m.running_mean.uniform_(-0.5, 0.5)
        m.running_var.uniform_(0.5, 2.0)
    m.eval()
    x = torch.randn(2, 6, 6, 6, 4)
    got = m(x)
    cs, ps = m.specs(tuple(x.shape))
    y = R.conv(x, m.weight, None, cs)
    z = torch.relu((y - m.running_mean) * torch.rsqrt(m.running_var + m.bn_eps) * m.gamma + m.beta)
    want = R.pool(z, ps, "max")
    torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-5)


def test_reference_ops_gradcheck_fp64():
    """torch.autograd.gradcheck (fp64) of the CPU oracle ops that the HIP kernels are tested against:
    strided / padded / dilated conv with bias + act, depthwise conv, avg + max pool, training-mode BN,
    label-smoothed softmax cross-entropy."""
    from torch.autograd import gradcheck

    from featurenet_amd.ops import reference as R
    from featurenet_amd.ops.spec import ConvSpec, PoolSpec

    torch.manual_seed(0)
    d = torch.float64
    x = torch.randn(2, 1, 7, 8, 3, dtype=d, requires_grad=True)
    for k, s, pad, dil, act in (((1, 3, 3), 1, "same", 1, "tanh"), ((1, 3, 1), 2, "valid", 1, None),
                                ((1, 3, 3), 1, "same", 2, "sigmoid")):
        spec = ConvSpec.make(x.shape, 4, k, s, pad, dil)
        w = torch.randn(4, spec.KD, spec.KH, spec.KW, 3, dtype=d, requires_grad=True)
        b = torch.randn(4, dtype=d, requires_grad=True)
        assert gradcheck(lambda x, w, b: R.conv(x, w, b, spec, act), (x, w, b))
    x3 = torch.randn(1, 4, 5, 6, 2, dtype=d, requires_grad=True)
    spec3 = ConvSpec.make(x3.shape, 3, (2, 2, 2), 1, "valid")
    w3 = torch.randn(3, 2, 2, 2, 2, dtype=d, requires_grad=True)
    assert gradcheck(lambda x, w: R.conv(x, w, None, spec3, "relu"), (x3, w3))
    dspec = ConvSpec.make(x.shape, 3, (1, 3, 3), 1, "same")
    wd = torch.randn(3, 1, 3, 3, 1, dtype=d, requires_grad=True)
    assert gradcheck(lambda x, w: R.depthwise_conv(x, w, None, dspec), (x, wd))
    ps = PoolSpec.make(x.shape, (1, 2, 2), (1, 2, 2), "same")
    assert gradcheck(lambda x: R.pool(x, ps, "avg"), (x,))
    xm = (torch.arange(2 * 7 * 8 * 3, dtype=d).reshape(2, 1, 7, 8, 3) % 17 / 17.0).requires_grad_(True)   # no ties
    assert gradcheck(lambda x: R.pool(x, ps, "max"), (xm,))
    g, be = torch.rand(3, dtype=d, requires_grad=True), torch.randn(3, dtype=d, requires_grad=True)
    rm, rv = torch.zeros(3, dtype=d), torch.ones(3, dtype=d)
    assert gradcheck(lambda x, g, be: R.batchnorm_act(x, g, be, rm.clone(), rv.clone(), True, 0.1, 1e-5, "tanh"),
                     (x, g, be))
    logits = torch.randn(5, 7, dtype=d, requires_grad=True)
    y = torch.randint(0, 7, (5,))
    assert gradcheck(lambda l: R.softmax_xent(l, y, 0.1), (logits,))


def test_conv_spec_extra_padding_equals_padded_input():
    """A ZeroPadding folded into the next conv (``ConvSpec.make(..., extra=...)``) computes the
    same as the conv over the explicitly padded input."""
    import torch

    from featurenet_amd.ops import reference as refops
    from featurenet_amd.ops.spec import ConvSpec

    torch.manual_seed(0)
    x = torch.randn(2, 1, 9, 11, 8)
    w = torch.randn(16, 1, 3, 3, 8)
    for padding in ("valid", "same"):
        xp = torch.nn.functional.pad(x, (0, 0, 2, 2, 1, 1))
        s_pad = ConvSpec.make(tuple(xp.shape), 16, (1, 3, 3), 1, padding)
        s_fold = ConvSpec.make(tuple(x.shape), 16, (1, 3, 3), 1, padding, extra=(0, 1, 2))
        assert (s_fold.OD, s_fold.OH, s_fold.OW) == (s_pad.OD, s_pad.OH, s_pad.OW)
        torch.testing.assert_close(refops.conv(x, w, None, s_fold), refops.conv(xp, w, None, s_pad))


@pytest.mark.parametrize("shape,k,s,pad", [((2, 12, 11, 13, 1), 7, 2, "same"), ((1, 10, 10, 10, 2), 4, 2, "same"),
                                           ((2, 13, 12, 11, 1), 7, 2, "valid")])
def test_s2d_padded_strided_conv_equals_direct(shape, k, s, pad):
    """Space-to-depth of the zero-padded input + the unpadded stride-1 conv over it == the
    padded strided conv (the seg model's 'same' 7^3 stride-2 stem takes this path)."""
    import importlib
    C = importlib.import_module("featurenet_amd.ops.conv")
    torch.manual_seed(3)
    x = torch.randn(*shape)
    spec = ConvSpec.make(x.shape, 16, k, s, pad)
    plan = C.s2d_plan(spec)
    assert plan is not None
    f, spec2 = plan
    w = torch.randn(16, k, k, k, shape[-1])
    x2 = C.s2d_input(x, f, spec2, (spec.pd, spec.ph, spec.pw))
    y2 = R.conv(x2, C.s2d_weight(w, f, spec, spec2), None, spec2)
    torch.testing.assert_close(y2, R.conv(x, w, None, spec), rtol=1e-4, atol=1e-4)


def test_pad_fold_rule_keeps_pads_beyond_the_kernel():
    """ZeroPadding folds into the next conv only while every total pad stays <= K - 1
    (the stride-1 dgrad runs with leading pads K - 1 - lo): a 1x1 conv after any padding,
    and a 'same' 3x3 after a fillSize-2 padding, keep the explicit pad op."""
    from featurenet_amd.ir.compile import _pad_foldable
    from featurenet_amd.models.layers import Conv

    assert _pad_foldable(Conv(8, 8, (1, 3, 3), 1, "valid"), (0, 1, 1))
    assert _pad_foldable(Conv(8, 8, (1, 3, 3), 1, "valid"), (0, 2, 2))
    assert _pad_foldable(Conv(8, 8, (1, 3, 3), 1, "same"), (0, 1, 1))
    assert not _pad_foldable(Conv(8, 8, (1, 3, 3), 1, "same"), (0, 2, 2))
    assert not _pad_foldable(Conv(8, 8, (1, 1, 1), 1, "valid"), (0, 1, 1))
    assert not _pad_foldable(Conv(8, 8, (1, 3, 3), 2, "valid"), (0, 1, 1))
    assert _pad_foldable(Conv(8, 8, (1, 5, 1), 1, "same"), (0, 2, 0))
    assert not _pad_foldable(Conv(8, 8, (1, 5, 1), 1, "same"), (0, 2, 1))


def test_flat_params_rebuild_releases_old_hooks():
    """A FlatParams built again on the same module supersedes the old one: the old one's
    hooks are removed (no pile-up, no reference keeping its buffers alive) and gradients
    land in the new flat buffer only."""
    import gc
    import weakref

    import torch
    from torch import nn

    from featurenet_amd.training.flat import FlatParams

    torch.manual_seed(0)
    m = nn.Sequential(nn.Linear(4, 3), nn.Linear(3, 2))
    f1 = FlatParams(m)
    ref1 = weakref.ref(f1)
    f2 = FlatParams(m)
    del f1
    gc.collect()
    assert ref1() is None, "the superseded FlatParams is still referenced (hooks left behind)"
    hooks = sum(len(p._post_accumulate_grad_hooks or {}) for p in m.parameters())
    assert hooks == len(list(m.parameters()))
    f2.zero_grad()
    x = torch.randn(5, 4)
    m(x).sum().backward()
    for p, off, n in f2.slices:
        assert p.grad.data_ptr() == f2.grad[off:off + n].data_ptr()
        assert torch.equal(f2.grad[off:off + n].view(p.shape), p.grad)
    assert f2.grad.abs().sum() > 0
