"""HIP kernel numerics vs the PyTorch fp32 reference of the same op.

Every test feeds identical bf16-rounded inputs to the native kernel and to
the fp32 reference (``featurenet_amd.ops.reference``) and compares with
tolerances scaled to bf16 output rounding.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

from featurenet_amd import _native  # noqa: E402
from featurenet_amd.ops import reference as ref  # noqa: E402
from featurenet_amd.ops.spec import ConvSpec, PoolSpec  # noqa: E402


def _native_loaded():
    assert _native.kernels_available(), "HIP kernel library (_C) must be built and loadable on the GPU box"


def close(a, b, rtol=2e-2, atol_frac=1e-2):
    a = a.float().cpu()
    b = b.float().cpu()
    scale = b.abs().max().item() + 1e-6
    err = (a - b).abs().max().item()
    assert err <= atol_frac * scale + rtol * 0, f"max abs err {err:.4g} vs scale {scale:.4g}"


CONV_CASES = [
    # (N, D, H, W, C, K, kernel, stride, padding)
    (2, 29, 29, 29, 32, 32, (5, 5, 5), 1, "valid"),      # FeatureNet conv2
    (2, 25, 25, 25, 32, 64, (4, 4, 4), 1, "valid"),      # conv3
    (2, 22, 22, 22, 64, 64, (3, 3, 3), 1, "valid"),      # conv4
    (2, 64, 64, 64, 1, 32, (7, 7, 7), 2, "valid"),       # conv1 (Cin=1 scalar gather)
    (4, 1, 32, 32, 3, 6, (1, 5, 5), 1, "same"),           # LeNet-style 2-D, odd channels
    (4, 1, 16, 16, 16, 24, (1, 3, 3), 2, "same"),         # strided same-padded 2-D
    (3, 1, 15, 17, 24, 100, (1, 3, 1), 1, "same"),        # asymmetric kernel, Cout > 64
    (5, 1, 1, 40, 8, 16, (1, 1, 5), 1, "same"),           # 1-D conv
    (2, 9, 10, 11, 16, 48, (3, 3, 3), 1, "same"),         # halo path: same padding, partial col block
    (2, 1, 20, 23, 48, 32, (1, 5, 5), 1, "same"),         # halo path: 2-D, 3 channel slices
    (1, 6, 7, 30, 32, 16, (2, 3, 3), 1, "valid"),         # halo path: even kernel, Cout 16
    (4, 1, 16, 16, 12, 120, (1, 5, 5), 1, "same"),        # LeNet conv3: split-K gather fwd + dgrad
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_bwd(case):
    _native_loaded()
    from featurenet_amd.ops.conv import ConvFn

    N, D, H, W, C, K, k, s, pad = case
    torch.manual_seed(0)
    dev = "cuda"
    x = torch.randn(N, D, H, W, C, device=dev).to(torch.bfloat16)
    spec = ConvSpec.make(x.shape, K, k, s, pad)
    w = (torch.randn(K, spec.KD, spec.KH, spec.KW, C, device=dev) * 0.05).to(torch.bfloat16).float()
    b = torch.randn(K, device=dev) * 0.1
    xr = x.float().clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    yr = ref.conv(xr, wr, br, spec)
    xn = x.clone().requires_grad_(True)
    wn = w.clone().requires_grad_(True)
    bn = b.clone().requires_grad_(True)
    yn, _ = ConvFn.apply(xn, wn, bn, spec, 0, False)
    assert yn.shape == yr.shape
    close(yn, yr)
    g = torch.randn_like(yr).to(torch.bfloat16).float()
    yr.backward(g)
    yn.backward(g.to(torch.bfloat16))
    close(xn.grad, xr.grad)
    close(wn.grad, wr.grad)
    close(bn.grad, br.grad)


def _search_space_shapes(n=18, seed=2024):
    """Random conv shapes from the reference search space (model/input.py:246-306 and the
    mutation tables, model/mutation/mutable_input.py): 2-D kernels from the 10 mutation
    shapes, 3-D cubes, stride 1/2, same/valid padding, channel counts 6..130 that are
    mostly NOT multiples of 16, occasional dilation (the combination projection)."""
    import random

    rng = random.Random(seed)
    k2d = [(1, 1), (3, 1), (1, 3), (3, 3), (5, 1), (1, 5), (5, 5), (7, 1), (1, 7), (7, 7)]
    out = []
    for i in range(n):
        three_d = i % 3 == 0
        cin = rng.choice([1, 3, 6, 8, 12, 16, 24, 30, 32, 48, 64, 96])
        cout = rng.choice([6, 12, 16, 25, 32, 40, 64, 100, 130])
        stride = rng.choice([1, 1, 2])
        pad = rng.choice(["same", "valid"])
        dil = 2 if (stride == 1 and rng.random() < 0.15) else 1
        if three_d:
            k = rng.choice([1, 3, 4, 5])
            size = rng.choice([9, 12, 16])
            shape, kern = (2, size, size + 1, size + 2, cin), (k, k, k)
        else:
            kh, kw = rng.choice(k2d)
            size = rng.choice([14, 28, 32])
            shape, kern = (3, 1, size, size + 3, cin), (1, kh, kw)
        out.append((shape, cout, kern, stride, pad, dil))
    return out


@pytest.mark.parametrize("case", _search_space_shapes())
def test_conv_search_space_shapes(case):
    """NAS shape generality: fwd / dgrad / wgrad / bias-grad through ConvFn vs the fp32 CPU oracle."""
    _native_loaded()
    from featurenet_amd.ops.conv import ConvFn

    shape, K, k, s, pad, dil = case
    torch.manual_seed(sum(shape) * 7 + K)
    x = torch.randn(*shape).to(torch.bfloat16)
    try:
        spec = ConvSpec.make(x.shape, K, k, s, pad, dil)
    except ValueError:
        pytest.skip("kernel larger than the input for this draw")
    if min(spec.OD, spec.OH, spec.OW) < 1:
        pytest.skip("empty output")
    w = (torch.randn(K, spec.KD, spec.KH, spec.KW, shape[-1]) * 0.1).to(torch.bfloat16).float()
    b = torch.randn(K) * 0.1
    xr, wr, br = x.float().clone().requires_grad_(True), w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = ref.conv(xr, wr, br, spec)
    xn = x.cuda().requires_grad_(True)
    wn, bn = w.cuda().requires_grad_(True), b.cuda().requires_grad_(True)
    yn, _ = ConvFn.apply(xn, wn, bn, spec, 0, False)
    assert yn.shape == yr.shape
    close(yn, yr)
    g = torch.randn_like(yr).to(torch.bfloat16).float()
    yr.backward(g)
    yn.backward(g.cuda().to(torch.bfloat16))
    close(xn.grad, xr.grad)
    close(wn.grad, wr.grad)
    close(bn.grad, br.grad)


@pytest.mark.parametrize("case", [
    # (x shape, Cout, kernel, stride, act): NAS channel counts that are not multiples of 8
    ((16, 1, 16, 16, 12), 120, (1, 5, 5), 1, "relu"),
    ((8, 1, 32, 32, 18), 108, (1, 3, 3), 1, "relu"),
    ((8, 1, 32, 32, 48), 12, (1, 5, 5), 1, None),
    ((4, 1, 8, 8, 36), 8, (1, 3, 3), 2, "relu"),
    ((6, 1, 28, 28, 20), 6, (1, 3, 1), 1, None),
    ((2, 9, 9, 9, 12), 20, (3, 3, 3), 1, "relu"),
])
def test_conv_channel_padded(case, monkeypatch):
    """C or Cout % 8 != 0: the forward gathers a channel-padded copy of x, the backward a
    channel-padded dy (16-B vectors instead of single elements); gradients cropped back."""
    _native_loaded()
    import importlib

    from featurenet_amd.ops.spec import act_code

    convmod = importlib.import_module("featurenet_amd.ops.conv")

    calls = []
    real = convmod.pad_channels
    monkeypatch.setattr(convmod, "pad_channels", lambda x, cp: calls.append((x.shape[-1], cp)) or real(x, cp))
    shape, K, k, s, act = case
    torch.manual_seed(K + shape[-1])
    x = torch.randn(*shape).to(torch.bfloat16)
    spec = ConvSpec.make(x.shape, K, k, s, "same")
    w = (torch.randn(K, spec.KD, spec.KH, spec.KW, shape[-1]) * 0.1).to(torch.bfloat16).float()
    b = torch.randn(K) * 0.1
    xr, wr, br = x.float().clone().requires_grad_(True), w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = ref.conv(xr, wr, br, spec, act)
    xn = x.cuda().requires_grad_(True)
    wn, bn = w.cuda().requires_grad_(True), b.cuda().requires_grad_(True)
    yn, _ = convmod.ConvFn.apply(xn, wn, bn, spec, act_code(act), False)
    close(yn, yr)
    g = torch.randn_like(yr).to(torch.bfloat16).float()
    yr.backward(g)
    yn.backward(g.cuda().to(torch.bfloat16))
    close(xn.grad, xr.grad)
    close(wn.grad, wr.grad)
    close(bn.grad, br.grad)
    assert wn.grad.shape == w.shape and xn.grad.shape == x.shape
    assert calls, "the channel-padded path did not run"


@pytest.mark.parametrize("case", [
    # LeNet-5 conv1 / conv2 (packed-W gather: C < 8), a channel-padded input (C = 12 -> 16) with
    # Cout % 8 != 0: (x shape, Cout, kernel, padding)
    ((16, 1, 32, 32, 3), 6, (1, 5, 5), "valid"),
    ((16, 1, 14, 14, 6), 16, (1, 5, 5), "valid"),
    ((4, 6, 7, 8, 5), 12, (1, 1, 7), "same"),
    ((8, 1, 20, 20, 12), 20, (1, 3, 1), "same"),
])
def test_conv_padded_wgrad_cropped_in_kernel(case, monkeypatch):
    """Weight gradients on the gather kernel written straight into the real [K, taps, C] shape:
    the epilogue drops the padding columns of the gather layout (packed-W rows, padded input
    channels) and reads the unpadded dy (no padded dy / dW copies, no fill, no crop copy) --
    same dW / db as the fp32 oracle."""
    _native_loaded()
    import importlib

    convmod = importlib.import_module("featurenet_amd.ops.conv")
    calls = []
    real = convmod.igemm_wgrad_cropped
    def counted(*a, **k):
        r = real(*a, **k)
        calls.append(r is not None)
        return r

    monkeypatch.setattr(convmod, "igemm_wgrad_cropped", counted)
    shape, K, k, pad = case
    torch.manual_seed(K * 3 + shape[-1])
    x = torch.randn(*shape).to(torch.bfloat16)
    spec = ConvSpec.make(x.shape, K, k, 1, pad)
    w = (torch.randn(K, spec.KD, spec.KH, spec.KW, shape[-1]) * 0.1).to(torch.bfloat16).float()
    b = torch.randn(K) * 0.1
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = ref.conv(x.float(), wr, br, spec, "relu")
    wn, bn = w.cuda().requires_grad_(True), b.cuda().requires_grad_(True)
    yn, _ = convmod.ConvFn.apply(x.cuda(), wn, bn, spec, 1, False)
    close(yn, yr)
    g = torch.randn_like(yr).to(torch.bfloat16).float()
    yr.backward(g)
    yn.backward(g.cuda().to(torch.bfloat16))
    close(wn.grad, wr.grad)
    close(bn.grad, br.grad)
    assert calls and all(calls), "the cropped weight-gradient path did not run"


@pytest.mark.parametrize("case", [
    ((2, 8, 8, 8, 32), 25, "none", True),       # segmentation classifier class: 32 -> 25 (+bias)
    ((4, 1, 14, 14, 24), 48, "relu", True),     # K % 8 == 0, N > 32
    ((2, 1, 8, 9, 6), 40, "none", False),       # 6 input channels: rows straddle 16-B chunks
    ((1, 4, 4, 4, 64), 64, "tanh", True),       # 64 x 64
])
def test_pointwise_conv(case):
    """1x1x1 convs on the streaming pointwise kernels (pointwise.hip): fwd + bias + act, dgrad, wgrad."""
    _native_loaded()
    from featurenet_amd.ops.conv import ConvFn, pointwise_ok
    from featurenet_amd.ops.spec import act_code

    shape, K, act, has_b = case
    torch.manual_seed(K)
    x = torch.randn(*shape).to(torch.bfloat16)
    spec = ConvSpec.make(x.shape, K, 1, 1)
    assert pointwise_ok(spec)
    w = (torch.randn(K, 1, 1, 1, shape[-1]) * 0.2).to(torch.bfloat16).float()
    b = torch.randn(K) * 0.1 if has_b else None
    a = None if act == "none" else act
    xr, wr = x.float().clone().requires_grad_(True), w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True) if has_b else None
    yr = ref.conv(xr, wr, br, spec, a)
    xn, wn = x.cuda().requires_grad_(True), w.cuda().requires_grad_(True)
    bn = b.cuda().requires_grad_(True) if has_b else None
    yn, _ = ConvFn.apply(xn, wn, bn, spec, act_code(a), False)
    close(yn, yr)
    g = torch.randn_like(yr).to(torch.bfloat16).float()
    yr.backward(g)
    yn.backward(g.cuda().to(torch.bfloat16))
    close(xn.grad, xr.grad)
    close(wn.grad, wr.grad)
    if has_b:
        close(bn.grad, br.grad)


def test_conv_stats_epilogue():
    _native_loaded()
    from featurenet_amd.ops.conv import native_conv_fwd, _pack_rows

    torch.manual_seed(1)
    x = torch.randn(2, 12, 12, 12, 32, device="cuda").to(torch.bfloat16)
    spec = ConvSpec.make(x.shape, 32, (3, 3, 3))
    w = torch.randn(32, 3, 3, 3, 32, device="cuda") * 0.05
    wm, ld = _pack_rows(w.reshape(32, -1))
    y, stats = native_conv_fwd(x, wm, ld, None, spec, 0, True)
    s = stats.sum(0)
    yf = y.float().reshape(-1, 32)
    torch.testing.assert_close(s[0], yf.sum(0), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(s[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("C,act", [(32, "relu"), (64, None), (6, "tanh"), (24, "sigmoid")])
@pytest.mark.parametrize("training", [True, False])
def test_batchnorm_act(C, act, training):
    _native_loaded()
    from featurenet_amd.ops.bn import batchnorm_act

    torch.manual_seed(2)
    y = (torch.randn(3, 5, 6, 7, C, device="cuda") * 2 + 0.5).to(torch.bfloat16)
    gamma = (torch.rand(C, device="cuda") + 0.5)
    beta = torch.randn(C, device="cuda") * 0.1
    rm, rv = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
    rm2, rv2 = rm.clone(), rv.clone()
    gr, br = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    yr = y.float().clone().requires_grad_(True)
    zr = ref.batchnorm_act(yr, gr, br, rm2, rv2, training, 0.1, 1e-5, act)
    gn, bn = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    yn = y.clone().requires_grad_(True)
    zn = batchnorm_act(yn, gn, bn, rm, rv, training, 0.1, 1e-5, act)
    close(zn, zr)
    if training:
        torch.testing.assert_close(rm, rm2, rtol=1e-3, atol=1e-4)
        torch.testing.assert_close(rv, rv2, rtol=1e-3, atol=1e-4)
    g = torch.randn_like(zr).to(torch.bfloat16).float()
    zr.backward(g)
    zn.backward(g.to(torch.bfloat16))
    close(yn.grad, yr.grad, atol_frac=2e-2)
    close(gn.grad, gr.grad)
    close(bn.grad, br.grad)


@pytest.mark.parametrize("shape,kernel,stride,pad,kind", [
    ((2, 20, 20, 20, 64), (2, 2, 2), None, "valid", "max"),
    ((3, 1, 9, 9, 16), (1, 3, 3), (1, 2, 2), "same", "max"),
    ((3, 1, 9, 9, 16), (1, 3, 3), (1, 1, 1), "same", "avg"),
    ((2, 1, 7, 7, 6), (1, 2, 2), None, "same", "avg"),
])
def test_pool(shape, kernel, stride, pad, kind):
    _native_loaded()
    from featurenet_amd.ops.pool import pool

    torch.manual_seed(3)
    x = torch.randn(*shape, device="cuda").to(torch.bfloat16)
    ps = PoolSpec.make(x.shape, kernel, stride, pad)
    # fp32 reference on the CPU: keeps the GPU library pooling out of the comparison
    xr = x.float().cpu().clone().requires_grad_(True)
    yr = ref.pool(xr, ps, kind)
    xn = x.clone().requires_grad_(True)
    yn = pool(xn, ps, kind)
    close(yn, yr)
    g = torch.randn_like(yr).to(torch.bfloat16).float()
    yr.backward(g)
    yn.backward(g.cuda().to(torch.bfloat16))
    close(xn.grad, xr.grad)


def test_bn_act_pool_fused():
    _native_loaded()
    from featurenet_amd.ops.bn import batchnorm_act_pool

    torch.manual_seed(4)
    C = 64
    y = torch.randn(2, 8, 8, 8, C, device="cuda").to(torch.bfloat16)
    ps = PoolSpec.make(y.shape, (2, 2, 2))
    g0, b0 = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    gr, br = g0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
    yr = y.float().clone().requires_grad_(True)
    zr = ref.pool(ref.batchnorm_act(yr, gr, br, rm.clone(), rv.clone(), True, 0.1, 1e-5, "relu"), ps, "max")
    gn, bn = g0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
    yn = y.clone().requires_grad_(True)
    zn = batchnorm_act_pool(yn, gn, bn, rm, rv, True, ps, "max", act="relu")
    close(zn, zr)
    g = torch.randn_like(zr).to(torch.bfloat16).float()
    zr.backward(g)
    zn.backward(g.to(torch.bfloat16))
    close(yn.grad, yr.grad, atol_frac=3e-2)
    close(gn.grad, gr.grad, atol_frac=2e-2)
    close(bn.grad, br.grad, atol_frac=2e-2)


def test_softmax_xent():
    _native_loaded()
    from featurenet_amd.ops.loss import softmax_xent

    torch.manual_seed(5)
    for B, NC in ((7, 24), (64, 100), (3, 2)):
        logits = torch.randn(B, NC, device="cuda") * 3
        labels = torch.randint(0, NC, (B,), device="cuda")
        lr_ = logits.clone().requires_grad_(True)
        l_ref = torch.nn.functional.cross_entropy(lr_, labels)
        l_ref.backward()
        ln_ = logits.clone().requires_grad_(True)
        l_nat, correct = softmax_xent(ln_, labels, with_correct=True)
        l_nat.backward()
        torch.testing.assert_close(l_nat, l_ref, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(ln_.grad, lr_.grad, rtol=1e-4, atol=1e-6)
        assert int(correct.sum()) == int((logits.argmax(-1) == labels).sum())


def test_softmax_xent_dense_bf16():
    """Per-voxel form: bf16 logits [N, D, H, W, NC] read directly, bf16 d(logits), partial-sum loss,
    label smoothing; vs the fp32 torch reference on the same (bf16-rounded) logits."""
    _native_loaded()
    from featurenet_amd.ops.loss import softmax_xent

    torch.manual_seed(6)
    for shape, NC, sm in (((2, 9, 10, 11), 25, 0.0), ((3, 7, 5, 4), 25, 0.1), ((50000,), 70, 0.0)):
        logits = (torch.randn(*shape, NC, device="cuda") * 3).to(torch.bfloat16)
        labels = torch.randint(0, NC, shape, device="cuda")
        lr_ = logits.float().reshape(-1, NC).clone().requires_grad_(True)
        l_ref = torch.nn.functional.cross_entropy(lr_, labels.reshape(-1), label_smoothing=sm)
        l_ref.backward()
        ln_ = logits.clone().requires_grad_(True)
        l_nat, correct = softmax_xent(ln_, labels, smoothing=sm, with_correct=True)
        l_nat.backward()
        assert ln_.grad.dtype == torch.bfloat16
        torch.testing.assert_close(l_nat, l_ref, rtol=1e-4, atol=1e-5)
        g = ln_.grad.float().reshape(-1, NC)
        assert (g - lr_.grad).abs().max().item() <= 1e-2 * lr_.grad.abs().max().item()
        assert int(correct.sum()) == int((logits.float().argmax(-1) == labels).sum())


@pytest.mark.parametrize("keras", [True, False])
def test_adam_flat(keras):
    _native_loaded()
    from featurenet_amd.ops.optim import FlatAdam

    torch.manual_seed(6)
    n = 10_001
    p = torch.randn(n, device="cuda")
    g = torch.randn(n, device="cuda")
    shadow = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    a = FlatAdam(p.clone(), g, lr=1e-2, keras_eps=keras, shadow=shadow)
    b = FlatAdam(p.clone().cpu(), g.cpu(), lr=1e-2, keras_eps=keras)
    for _ in range(3):
        a.step(0.5)
        b.step(0.5)
    torch.testing.assert_close(a.p.cpu(), b.p, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(shadow.float().cpu(), b.p.bfloat16().float(), rtol=1e-2, atol=1e-3)


def test_dropout_mask_consistent():
    _native_loaded()
    from featurenet_amd.ops.elementwise import dropout

    x = torch.ones(4096, 32, device="cuda", dtype=torch.bfloat16).requires_grad_(True)
    y = dropout(x, 0.3, True)
    keep = (y.float() != 0)
    frac = keep.float().mean().item()
    assert 0.65 < frac < 0.75
    y.float().sum().backward()
    assert torch.equal(x.grad.float() != 0, keep)
    torch.testing.assert_close(y.float()[keep], torch.full_like(y.float()[keep], 1 / 0.7), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("bn", [False, True])
def test_featurenet3d_matches_reference_step(bn):
    """One full fwd/bwd of FeatureNet-3D on GPU (bf16 activations) vs the CPU fp32 reference path.

    The two paths differ by bf16 rounding of activations / weights; through a
    ReLU every pre-activation within rounding distance of 0 can flip its mask,
    and each flip moves a whole gradient entry, so the relative L2 error grows
    like sqrt(flip fraction) (~5-12 % here, largest at the first layer) while
    the gradient direction stays aligned.  Train-mode BN at batch 8 adds the
    cancellation of its mean terms.  Per-op numerics are asserted tightly in
    the tests above; this test guards the composition (cosine + L2 drift), and
    ``test_featurenet3d_per_layer_oracle_64cube`` bounds every layer at 2e-2.
    Measured (round 6; the step is bitwise repeatable, so these are the values on any box):
    without BN rel <= 0.122, cos >= 0.9926; with BN rel <= 0.237, cos >= 0.9731 (conv1's beta).
    """
    _native_loaded()
    from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig
    from featurenet_amd.ops import softmax_xent

    torch.manual_seed(7)
    cfg = FeatureNet3DConfig(input_size=32, num_classes=24, kernels=(5, 3, 3, 3), strides=(2, 1, 1, 1), bn=bn)
    m_gpu = FeatureNet3D(cfg)
    m_cpu = FeatureNet3D(cfg)
    m_cpu.load_state_dict(m_gpu.state_dict())
    m_gpu = m_gpu.cuda()
    x = (torch.rand(8, 32, 32, 32, 1) < 0.3).float()
    y = torch.randint(0, 24, (8,))
    lg = m_gpu(x.cuda().bfloat16())
    lc = m_cpu(x)
    close(lg, lc, atol_frac=5e-2)
    softmax_xent(lg, y.cuda()).backward()
    softmax_xent(lc, y).backward()
    report = []
    for (n1, p1), (n2, p2) in zip(m_gpu.named_parameters(), m_cpu.named_parameters()):
        a, b = p1.grad.float().cpu(), p2.grad.float()
        rel = ((a - b).norm() / (b.norm() + 1e-12)).item()
        cos = torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()
        report.append((n1, rel, cos))
    print("\n".join(f"{n:24s} rel={r:.4f} cos={c:.5f}" for n, r, c in report))
    for n, r, c in report:
        if bn:
            assert c > 0.97 and r < 0.28, f"{n}: rel={r:.3g} cos={c:.4f}"
        else:
            assert c > 0.99 and r < 0.15, f"{n}: rel={r:.3g} cos={c:.4f}"


HALO_CASES = [
    # (N, D, H, W, C, K, kernel, padding, act)
    (2, 29, 29, 29, 32, 32, (5, 5, 5), "valid", 0),
    (2, 25, 25, 25, 32, 64, (4, 4, 4), "valid", 0),
    (2, 22, 22, 22, 64, 64, (3, 3, 3), "valid", 0),
    (3, 7, 9, 12, 16, 48, (3, 3, 3), "same", 1),
    (2, 1, 31, 33, 32, 96, (1, 3, 3), "same", 2),
    (2, 10, 11, 12, 32, 32, (3, 3, 3), "same", 0),    # 27 taps, Cout 32: wgrad with half the taps per wave
    (1, 6, 6, 61, 32, 32, (5, 5, 5), "valid", 0),     # 57-wide output: W-split tiles (TW < OW)
    (1, 7, 5, 70, 32, 64, (3, 3, 3), "same", 1),       # W split with padding, BN = 64
]


@pytest.mark.parametrize("case", HALO_CASES)
def test_conv_halo_fwd_dgrad_stats(case):
    """LDS-halo kernel (conv_halo.hip): forward (+bias/act), BN-stats epilogue and dgrad."""
    _native_loaded()
    import importlib

    C = importlib.import_module("featurenet_amd.ops.conv")

    N, D, H, W, Ci, K, k, pad, act = case
    torch.manual_seed(3)
    x = torch.randn(N, D, H, W, Ci, device="cuda").to(torch.bfloat16)
    spec = C.ConvSpec.make(x.shape, K, k, 1, pad)
    assert C.halo_fwd_plan(spec) is not None and C.halo_dgrad_plan(spec) is not None
    if W >= 61:
        assert C.halo_fwd_plan(spec)[2] < spec.OW, C.halo_fwd_plan(spec)     # the case really splits W
    w = (torch.randn(K, spec.KD, spec.KH, spec.KW, Ci, device="cuda") * 0.05).to(torch.bfloat16).float()
    b = torch.randn(K, device="cuda") * 0.1
    acts = {0: None, 1: "relu", 2: "tanh"}
    y, _ = C.halo_conv_fwd(x, w, b, spec, act, False, C.halo_fwd_plan(spec))
    yr = ref.conv(x.float(), w, b, spec, acts[act])
    close(y, yr)
    if act == 0:
        y2, st = C.halo_conv_fwd(x, w, None, spec, 0, True, C.halo_fwd_plan(spec))
        yr2 = ref.conv(x.float(), w, None, spec).reshape(-1, K)
        yb = y2.float().reshape(-1, K)
        torch.testing.assert_close(st[:, 0].sum(0), yb.sum(0), rtol=2e-3, atol=2e-2)
        torch.testing.assert_close(st[:, 1].sum(0), (yb * yb).sum(0), rtol=2e-3, atol=2e-2)
        close(y2.reshape(-1, K), yr2)
    g = (torch.randn(spec.out_shape5, device="cuda")).to(torch.bfloat16)
    dx = C.halo_conv_dgrad(g, w, spec, C.halo_dgrad_plan(spec))
    xr = x.float().clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    ref.conv(xr, wr, None, spec).backward(g.float())
    close(dx, xr.grad)
    if C.halo_wgrad_plan(spec) is not None:
        dw = C.halo_conv_wgrad(g, x, spec, C.halo_wgrad_plan(spec))
        close(dw, wr.grad)


def test_halo_schedule_counters_reset_and_repeatable():
    """The dynamic tile schedule leaves its counters zero after every launch (the last
    workgroup out resets them), so back-to-back launches and graph replays start clean;
    the result does not depend on which workgroup took which tile."""
    _native_loaded()
    import importlib

    C = importlib.import_module("featurenet_amd.ops.conv")
    torch.manual_seed(12)
    x = torch.randn(2, 20, 21, 22, 32, device="cuda").to(torch.bfloat16)
    spec = ConvSpec.make(x.shape, 64, (3, 3, 3), 1, "same")
    w = (torch.randn(64, 3, 3, 3, 32, device="cuda") * 0.05).to(torch.bfloat16).float()
    st = torch.cuda.current_stream().cuda_stream
    outs, dws = [], []
    for _ in range(3):
        y, stats = C.halo_conv_fwd(x, w, None, spec, 0, True, C.halo_fwd_plan(spec))
        dw = C.halo_conv_wgrad(y.contiguous(), x, spec, C.halo_wgrad_plan(spec))
        torch.cuda.synchronize()
        assert int(C.halo_sched(x.device, st).abs().sum()) == 0
        outs.append(y)
        dws.append(dw)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    torch.testing.assert_close(dws[0], dws[2], rtol=1e-5, atol=1e-4)   # fp32 atomics: order may differ


@pytest.mark.parametrize("case", [
    (2, 9, 10, 11, 8, 32, (3, 3, 3), "same"),       # 8-channel halo slices (CS = 8), partial taps
    (2, 12, 12, 12, 8, 64, (4, 4, 4), "valid"),     # s2d-stem shape class, BN = 64
    (2, 12, 12, 12, 8, 32, (4, 4, 4), "valid"),     # s2d stem, BN = 32: weights resident in LDS (4 stages)
    (3, 1, 17, 19, 24, 16, (1, 5, 5), "same"),      # C % 16 != 0 -> three 8-channel slices
])
def test_conv_halo_cs8(case):
    """Halo kernels with 8-channel slices: forward + BN stats and wgrad (ConvFn) vs fp32 reference."""
    _native_loaded()
    import importlib

    C = importlib.import_module("featurenet_amd.ops.conv")
    N, D, H, W, Ci, K, k, pad = case
    torch.manual_seed(11)
    x = torch.randn(N, D, H, W, Ci, device="cuda").to(torch.bfloat16)
    spec = ConvSpec.make(x.shape, K, k, 1, pad)
    assert C.halo_cs(Ci) == 8 and C.halo_fwd_plan(spec) is not None and C.halo_wgrad_plan(spec) is not None
    w = (torch.randn(K, spec.KD, spec.KH, spec.KW, Ci, device="cuda") * 0.05).to(torch.bfloat16).float()
    wn = w.clone().requires_grad_(True)
    y, st = C.ConvFn.apply(x, wn, None, spec, 0, True)
    wr = w.clone().requires_grad_(True)
    yr = ref.conv(x.float(), wr, None, spec)
    close(y, yr)
    yb = y.float().reshape(-1, K)
    torch.testing.assert_close(st[:, 0].sum(0), yb.sum(0), rtol=2e-3, atol=5e-2)
    g = torch.randn_like(yr).to(torch.bfloat16)
    y.backward(g)
    yr.backward(g.float())
    close(wn.grad, wr.grad)


def test_s2d_pack_matches_reference_layout():
    """s2d_pack kernel == the torch view/permute definition of the space-to-depth layout."""
    _native_loaded()
    import importlib

    C = importlib.import_module("featurenet_amd.ops.conv")
    torch.manual_seed(4)
    for shape, k, s, pad in (((2, 19, 20, 21, 1), 7, 2, "valid"), ((1, 9, 9, 9, 2), 4, 2, "valid"),
                             ((2, 20, 18, 22, 1), 7, 2, "same")):
        x = torch.randn(*shape, device="cuda").to(torch.bfloat16)
        spec = ConvSpec.make(x.shape, 16, k, s, pad)
        plan = C.s2d_plan(spec)
        if plan is None:
            continue
        f, spec2 = plan
        pads = (spec.pd, spec.ph, spec.pw)
        got = C.s2d_input(x, f, spec2, pads)
        want = C.s2d_input(x.cpu(), f, spec2, pads)
        assert torch.equal(got.cpu(), want)


DW_CASES = [
    # (N, D, H, W, C, kernel, stride, padding, act)
    (4, 1, 16, 16, 16, (1, 3, 3), 1, "same", "relu"),
    (2, 1, 15, 13, 3, (1, 5, 5), 2, "same", None),
    (2, 6, 7, 8, 8, (3, 3, 3), 1, "valid", "tanh"),
]


@pytest.mark.parametrize("case", DW_CASES)
def test_depthwise_fwd_bwd(case):
    """Depthwise kernels (dwconv.hip) vs the grouped-conv fp32 reference."""
    _native_loaded()
    from featurenet_amd.ops.conv import DepthwiseFn
    from featurenet_amd.ops.spec import act_code

    N, D, H, W, C, k, s, pad, act = case
    torch.manual_seed(5)
    x = torch.randn(N, D, H, W, C, device="cuda").to(torch.bfloat16)
    spec = ConvSpec.make(x.shape, C, k, s, pad)
    w = (torch.randn(C, spec.KD, spec.KH, spec.KW, 1, device="cuda") * 0.2).to(torch.bfloat16).float()
    b = torch.randn(C, device="cuda") * 0.1
    xr, wr, br = (t.float().clone().requires_grad_(True) for t in (x, w, b))
    yr = ref.depthwise_conv(xr, wr, br, spec, 1, act)
    xn, wn, bn = (t.clone().requires_grad_(True) for t in (x, w, b))
    yn = DepthwiseFn.apply(xn, wn, bn, spec, act_code(act))
    close(yn, yr)
    g = torch.randn_like(yr).to(torch.bfloat16).float()
    yr.backward(g)
    yn.backward(g.to(torch.bfloat16))
    close(xn.grad, xr.grad)
    close(wn.grad, wr.grad)
    close(bn.grad, br.grad)


def test_segmentation_head_step():
    """FeatureNet-3D-Seg (same-padded halo convs, x2 upsample, per-voxel loss) vs the fp32 CPU oracle."""
    _native_loaded()
    from featurenet_amd.models.featurenet3d import FeatureNet3DSeg
    from featurenet_amd.ops import softmax_xent

    torch.manual_seed(0)
    m_cpu = FeatureNet3DSeg(input_size=32, num_classes=5)
    m_gpu = FeatureNet3DSeg(input_size=32, num_classes=5).cuda()
    m_gpu.load_state_dict(m_cpu.state_dict())
    x = (torch.rand(2, 32, 32, 32, 1) < 0.3).float()
    y = torch.randint(0, 5, (2, 32, 32, 32))
    lc = softmax_xent(m_cpu(x), y)
    lg = softmax_xent(m_gpu(x.cuda().to(torch.bfloat16)), y.cuda())
    assert torch.isfinite(lg)
    assert abs(lg.item() - lc.item()) / lc.item() < 0.05
    lg.backward()
    for p in m_gpu.parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all()


@pytest.mark.parametrize("kernel", ["tile", "halo"])
@pytest.mark.parametrize("cin,cout,k,dims,out_f8", [
    (32, 64, 3, (2, 12, 13, 14), False),
    (32, 64, 3, (2, 12, 13, 14), True),
    (32, 32, 5, (4, 21, 20, 19), True),       # conv2-like: CS = 32, 4 taps per 128-k step, edge tiles
    (64, 64, 3, (3, 18, 17, 20), False),      # conv4-like: CS = 64, 2 taps per step
    (64, 64, 4, (2, 16, 16, 16), True),       # conv3-like tap count (64 -> pads the last step)
])
def test_conv_fp8(monkeypatch, kernel, cin, cout, k, dims, out_f8):
    """fp8 conv -- the F8 tile kernel (conv_tile.hip) or the fp8 halo kernel (conv_fp8.hip) --
    vs the fp32 conv of the same dequantised operands."""
    _native_loaded()
    from featurenet_amd.inference.fp8 import Fp8Conv
    from featurenet_amd.models.layers import Conv

    monkeypatch.setenv("FN_F8_TILE", "1" if kernel == "tile" else "0")
    torch.manual_seed(7)
    conv = Conv(cin, cout, (k, k, k), 1, "valid", bias=True).cuda()
    with torch.no_grad():
        conv.bias.normal_(0, 0.1)
    xs = 0.02
    x = (torch.randn(*dims, cin, device="cuda") * 2).clamp(-400 * xs, 400 * xs)
    xq = (x / xs).to(torch.float8_e4m3fn)
    out_scale = 0.05 if out_f8 else None
    layer = Fp8Conv(conv, xs, out_scale, relu=True)
    spec = ConvSpec.make(x.shape, cout, (k, k, k))
    if kernel == "tile":
        assert layer.tile_plan(spec) is not None, spec
    y, _ = layer(xq.view(torch.uint8), tuple(x.shape))
    yr = torch.relu(ref.conv(xq.float() * xs, layer.w_dequant, layer.bias, spec))
    if out_f8:
        yd = y.view(torch.float8_e4m3fn).float() * out_scale
        err = (yd - yr).abs().max().item()
        assert err <= 0.07 * yr.abs().max().item() + 2 * out_scale
    else:
        close(y, yr)


def test_fp8_featurenet3d_matches_bf16():
    _native_loaded()
    from featurenet_amd.inference.fp8 import quantize_model
    from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig

    torch.manual_seed(0)
    m = FeatureNet3D(FeatureNet3DConfig(input_size=32, num_classes=24)).cuda().eval()
    x = (torch.rand(16, 32, 32, 32, 1, device="cuda") < 0.3).to(torch.bfloat16)
    q = quantize_model(m, x[:8])
    with torch.no_grad():
        ref_logits = m(x).float()
        got = q(x).float()
    cos = torch.nn.functional.cosine_similarity(got.flatten(), ref_logits.flatten(), dim=0).item()
    assert cos > 0.97, cos


@pytest.mark.parametrize("padding", ["valid", "same"])
def test_space_to_depth_stem_matches_reference(padding):
    """FeatureNet-3D stem (1-ch 7^3 stride 2) through space-to-depth + halo kernels: fwd, stats, wgrad."""
    _native_loaded()
    import importlib

    C = importlib.import_module("featurenet_amd.ops.conv")
    torch.manual_seed(2)
    x = (torch.rand(2, 64, 64, 64, 1, device="cuda") < 0.3).to(torch.bfloat16)
    spec = ConvSpec.make(x.shape, 32, 7, 2, padding)
    assert C.s2d_plan(spec) is not None
    w = (torch.randn(32, 7, 7, 7, 1, device="cuda") * 0.05).to(torch.bfloat16).float()
    wn = w.clone().requires_grad_(True)
    y, st = C.ConvFn.apply(x, wn, None, spec, 0, True)
    wr = w.clone().requires_grad_(True)
    yr = ref.conv(x.float(), wr, None, spec)
    close(y, yr)
    yb = y.float().reshape(-1, 32)
    torch.testing.assert_close(st[:, 0].sum(0), yb.sum(0), rtol=2e-3, atol=5e-2)
    g = torch.randn_like(yr).to(torch.bfloat16)
    y.backward(g)
    yr.backward(g.float())
    close(wn.grad, wr.grad)


def test_graph_captured_training_matches_eager():
    """hipGraph-captured train step (fwd + bwd + device-state Adam) follows the eager trajectory."""
    _native_loaded()
    import time

    from featurenet_amd.ir.compile import compile_model
    from featurenet_amd.ir.parse import parse_feature_model
    from featurenet_amd.training.trainer import Trainer

    torch.manual_seed(0)
    x = torch.rand(64 * 12, 28, 28, 1, device="cuda")
    y = torch.randint(0, 10, (64 * 12,), device="cuda")
    res = {}
    for graph in (False, True):
        torch.manual_seed(1)
        net = compile_model(parse_feature_model("lenet5", name="l"), (28, 28, 1), 10)
        tr = Trainer(net, lr=1e-3, device="cuda", graph=graph)
        assert tr.graph_mode == graph
        losses = []
        for i in range(12):
            l, _ = tr.train_step(x[i * 64:(i + 1) * 64], y[i * 64:(i + 1) * 64])
            losses.append(float(l))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(50):
            tr.train_step(x[:64], y[:64])
        torch.cuda.synchronize()
        res[graph] = (losses, (time.perf_counter() - t0) / 50, tr.opt.t)
    le, lg = res[False][0], res[True][0]
    assert max(abs(a - b) for a, b in zip(le, lg)) < 2e-2 * max(abs(v) for v in le)
    assert res[True][2] == res[False][2] == 62
    print(f"\\nstep time eager {res[False][1] * 1e3:.3f} ms, graph {res[True][1] * 1e3:.3f} ms")


@pytest.mark.parametrize("K,C,k", [(32, 32, 5), (64, 32, 4), (16, 24, 3), (32, 8, 4)])
def test_halo_pack_weights_matches_torch_layout(K, C, k):
    """halo_pack_w kernel == the torch reference packing (forward and flipped/transposed dgrad layouts)."""
    _native_loaded()
    import importlib

    Cm = importlib.import_module("featurenet_amd.ops.conv")
    torch.manual_seed(9)
    spec = ConvSpec.make((1, 9, 9, 9, C), K, k)
    w = torch.randn(K, k, k, k, C, device="cuda")
    w3 = w.reshape(K, spec.taps, C)
    torch.testing.assert_close(Cm.halo_pack(w, spec, dgrad=False), Cm.halo_weights(w3), rtol=0, atol=0)
    if K % 8 == 0:
        ref_d = Cm.halo_weights(w3.flip(1).permute(2, 1, 0))
        torch.testing.assert_close(Cm.halo_pack(w, spec, dgrad=True), ref_d, rtol=0, atol=0)


@pytest.mark.parametrize("C", [16, 64, 24, 256, 8])
def test_upsample2x_fwd_bwd(C):
    """Nearest x2 upsample kernels vs the torch expand/reshape reference (fwd exact, bwd block
    sums); C / 8 a power of two <= 32 takes the output-row-major kernels, 24 the general ones."""
    _native_loaded()
    from featurenet_amd.ops.elementwise import upsample2x

    torch.manual_seed(9)
    x = torch.randn(2, 3, 4, 5, C, device="cuda").to(torch.bfloat16)
    xn = x.clone().requires_grad_(True)
    y = upsample2x(xn)
    n, d, h, w, c = x.shape
    ref_y = x.reshape(n, d, 1, h, 1, w, 1, c).expand(n, d, 2, h, 2, w, 2, c).reshape(n, 2 * d, 2 * h, 2 * w, c)
    assert torch.equal(y, ref_y)
    g = torch.randn_like(y.float()).to(torch.bfloat16)
    y.backward(g)
    ref_g = g.float().reshape(n, d, 2, h, 2, w, 2, c).sum((2, 4, 6))
    torch.testing.assert_close(xn.grad.float(), ref_g, rtol=1e-2, atol=2e-2)


def test_s2d_weight_map_matches_reference():
    """Native space-to-depth weight expand / gradient fold == the torch pad+permute reference."""
    import importlib

    cv = importlib.import_module("featurenet_amd.ops.conv")
    spec = ConvSpec.make((2, 64, 64, 64, 1), 32, (7, 7, 7), 2, "valid")
    f, spec2 = cv.s2d_plan(spec)
    torch.manual_seed(0)
    w = torch.randn(32, 7, 7, 7, 1)
    ref_w2 = cv.s2d_weight(w, f, spec, spec2)                 # CPU: torch reference path
    w2 = cv.s2d_weight(w.cuda(), f, spec, spec2)
    assert torch.equal(w2.cpu(), ref_w2)
    g2 = torch.randn_like(ref_w2)
    ref_g = cv.s2d_weight_grad(g2, f, spec)
    out = torch.zeros(32, 7, 7, 7, 1, device="cuda")
    g = cv.s2d_weight_grad(g2.cuda(), f, spec, out=out)
    assert g.data_ptr() == out.data_ptr() and torch.equal(g.cpu(), ref_g)


@pytest.mark.parametrize("M,K,N,act,bias", [(128, 64000, 128, "relu", True), (128, 128, 24, None, True),
                                            (64, 2048, 256, "relu", False), (96, 520, 64, None, True),
                                            (32, 4096, 512, "relu", True), (64, 120, 84, "relu", True),
                                            (64, 84, 10, None, True), (96, 400, 10, None, False),
                                            (50, 84, 10, "relu", True), (20, 30, 7, None, True),
                                            (1024, 400, 120, "relu", True), (700, 84, 10, None, True)])
def test_dense_native_matches_fp32(M, K, N, act, bias):
    """Native Dense (split-K forward, dgrad, fp32 wgrad/db) vs the fp32 PyTorch reference."""
    from featurenet_amd.ops.linear import LinearFn

    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).requires_grad_(True)
    b = (torch.randn(N, device="cuda") * 0.1).requires_grad_(True) if bias else None
    xg = x.clone().requires_grad_(True)
    from featurenet_amd.ops.spec import act_code

    y = LinearFn.apply(xg, w, b, act_code(act), False)
    wr = w.detach().to(torch.bfloat16).float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True) if bias else None
    xr = x.float().requires_grad_(True)
    yr = xr @ wr.t() + (br if bias else 0)
    if act == "relu":
        yr = torch.relu(yr)
    l2 = ((y.float() - yr).norm() / yr.norm()).item()
    assert l2 < 1e-2, l2
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    gx, gw, *gb = torch.autograd.grad(y, [xg, w] + ([b] if bias else []), dy)
    rx, rw, *rb = torch.autograd.grad(yr, [xr, wr] + ([br] if bias else []), dy.float())
    for a, r_ in [(gx, rx), (gw, rw)] + ([(gb[0], rb[0])] if bias else []):
        e = ((a.float() - r_).norm() / (r_.norm() + 1e-12)).item()
        assert e < 2e-2, e


@pytest.mark.parametrize("M,K,N,act", [(1024, 140608, 128, "relu"), (128, 64000, 128, None), (64, 84, 10, None),
                                        (300, 520, 200, "relu"), (33, 4096, 64, None)])
def test_dense_infer_bf16_weights(M, K, N, act):
    """Inference Dense on a bf16 weight copy (128-column workgroups when N > 64) vs fp32 PyTorch."""
    from featurenet_amd.ops.linear import linear_infer

    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda") * 0.1
    y = linear_infer(x, w, b, act, out_fp32=True)
    yr = x.float() @ w.float().t() + b
    if act == "relu":
        yr = torch.relu(yr)
    assert y.dtype == torch.float32 and y.shape == (M, N)
    assert ((y - yr).norm() / yr.norm()).item() < 1e-4


@pytest.mark.parametrize("shape", [(2, 3, 5, 7, 16), (3, 1, 4, 6, 5)])
def test_combine_kernels_match_torch(shape):
    """Native add / multiply (+fused backward), two-way concat (+split) and zero padding
    (+crop) vs torch on bf16 channels-last tensors (vector and scalar paths)."""
    from featurenet_amd.ops import elementwise as ew

    torch.manual_seed(0)
    a = torch.randn(shape, device="cuda").to(torch.bfloat16).requires_grad_(True)
    b = torch.randn(shape, device="cuda").to(torch.bfloat16).requires_grad_(True)
    g = torch.randn(shape, device="cuda").to(torch.bfloat16)
    for fn, ref_fn in ((ew.add, torch.add), (ew.multiply, torch.mul)):
        y = fn(a, b)
        assert torch.equal(y, ref_fn(a.detach(), b.detach()))
        ga, gb = torch.autograd.grad(y, [a, b], g)
        ra, rb = torch.autograd.grad(ref_fn(a, b), [a, b], g)
        assert torch.equal(ga, ra) and torch.equal(gb, rb)
    for ax in (1, 4):
        y = ew.concat([a, b], ax)
        assert torch.equal(y, torch.cat([a.detach(), b.detach()], ax))
        gy = torch.randn(y.shape, device="cuda").to(torch.bfloat16)
        ga, gb = torch.autograd.grad(y, [a, b], gy)
        assert torch.equal(ga, gy.narrow(ax, 0, shape[ax])) and torch.equal(gb, gy.narrow(ax, shape[ax], shape[ax]))
    y = ew.zero_pad(a, (1, 2, 0))
    ref = torch.nn.functional.pad(a.detach(), (0, 0, 0, 0, 2, 2, 1, 1))
    assert torch.equal(y, ref)
    gy = torch.randn(y.shape, device="cuda").to(torch.bfloat16)
    (ga,) = torch.autograd.grad(y, [a], gy)
    assert torch.equal(ga, gy[:, 1:-1, 2:-2, :, :])


def test_featurenet3d_training_trajectory_matches_fp32():
    """10 Adam steps of FeatureNet-3D (32^3, BN) on the native bf16 GPU path vs the fp32 CPU
    reference path from the same init on fixed, learnable data (label = the octant holding
    the most occupied voxels): both loss curves fall and stay within a bf16 band."""
    _native_loaded()
    from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig
    from featurenet_amd.ops import FlatAdam, softmax_xent
    from featurenet_amd.training.flat import FlatParams

    torch.manual_seed(3)
    cfg = FeatureNet3DConfig(input_size=32, num_classes=8, kernels=(5, 3, 3, 3), strides=(2, 1, 1, 1), fc=64)
    m_gpu, m_cpu = FeatureNet3D(cfg), FeatureNet3D(cfg)
    m_cpu.load_state_dict(m_gpu.state_dict())
    m_gpu = m_gpu.cuda()
    g = torch.Generator().manual_seed(11)
    x = (torch.rand(32, 32, 32, 32, 1, generator=g) < 0.15).float()
    octant = torch.zeros(32, 8)
    for i in range(8):
        d, h, w = (i >> 2) & 1, (i >> 1) & 1, i & 1
        sl = x[:, d * 16:(d + 1) * 16, h * 16:(h + 1) * 16, w * 16:(w + 1) * 16]
        octant[:, i] = sl.sum(dim=(1, 2, 3, 4))
    for n in range(32):                          # make the label octant clearly denser
        i = n % 8
        d, h, w = (i >> 2) & 1, (i >> 1) & 1, i & 1
        x[n, d * 16:(d + 1) * 16, h * 16:(h + 1) * 16, w * 16:(w + 1) * 16] = \
            (torch.rand(16, 16, 16, 1, generator=g) < 0.45).float()
    y = torch.arange(32) % 8
    curves = []
    for model, dev, xin in ((m_gpu, "cuda", x.cuda().bfloat16()), (m_cpu, "cpu", x)):
        flat = FlatParams(model)
        opt = FlatAdam(flat.data, flat.grad, lr=3e-4)
        yy = y.to(dev)
        losses = []
        for _ in range(10):
            flat.zero_grad()
            loss = softmax_xent(model(xin), yy)
            loss.backward()
            opt.step()
            losses.append(float(loss.detach()))
        curves.append(losses)
    gpu, cpu = curves
    print("gpu", [round(v, 3) for v in gpu])
    print("cpu", [round(v, 3) for v in cpu])
    assert gpu[-1] < 0.7 * gpu[0] and cpu[-1] < 0.7 * cpu[0], (gpu, cpu)
    # BN at batch 32 + Adam amplify bf16 differences in the transient; the band is relative
    # to the larger of the two losses (a round-1 blow-up would miss it by orders of magnitude)
    for a, b in zip(gpu, cpu):
        assert abs(a - b) < 0.1 + 0.25 * max(a, b), (gpu, cpu)


@pytest.mark.parametrize("k,padding,extra", [((1, 3, 3), "valid", (0, 1, 1)), ((1, 3, 3), "valid", (0, 2, 2)),
                                             ((1, 3, 3), "same", (0, 1, 1)), ((1, 5, 1), "same", (0, 2, 0)),
                                             ((3, 3, 3), "valid", (0, 1, 2))])
@pytest.mark.parametrize("C,K", [(16, 32), (6, 12)])
def test_folded_zero_padding_matches_explicit_pad(k, padding, extra, C, K):
    """A ZeroPadding folded into the next conv (ConvSpec extra pads, ir/compile.py fold_pads)
    gives the same forward, dx and dW on the native kernels as the explicit pad followed by
    the conv (every extra pad here is one the fold rule accepts: total pad <= K - 1)."""
    _native_loaded()
    from featurenet_amd.ir.compile import _pad_foldable
    from featurenet_amd.models.layers import Conv
    from featurenet_amd.ops.conv import ConvFn

    assert _pad_foldable(Conv(C, K, k, 1, padding), extra)
    torch.manual_seed(5)
    x = torch.randn(2, 6, 13, 14, C, device="cuda").to(torch.bfloat16)
    ed, eh, ew = extra
    xp = torch.nn.functional.pad(x.float(), (0, 0, ew, ew, eh, eh, ed, ed)).to(torch.bfloat16)
    s_fold = ConvSpec.make(tuple(x.shape), K, k, 1, padding, extra=extra)
    s_pad = ConvSpec.make(tuple(xp.shape), K, k, 1, padding)
    w = (torch.randn(K, *k, C, device="cuda") * 0.05).to(torch.bfloat16).float()
    xa = x.clone().requires_grad_(True)
    wa = w.clone().requires_grad_(True)
    ya, _ = ConvFn.apply(xa, wa, None, s_fold, 0, False)
    xb = xp.clone().requires_grad_(True)
    wb = w.clone().requires_grad_(True)
    yb, _ = ConvFn.apply(xb, wb, None, s_pad, 0, False)
    assert ya.shape == yb.shape
    close(ya, yb)
    g = torch.randn_like(yb.float()).to(torch.bfloat16)
    ya.backward(g)
    yb.backward(g)
    dx_ref = xb.grad.float()[:, ed:ed + x.shape[1], eh:eh + x.shape[2], ew:ew + x.shape[3]]
    close(xa.grad, dx_ref)
    close(wa.grad, wb.grad)


def test_featurenet3d_per_layer_oracle_64cube():
    """Composition oracle at the production input (64^3, batch 32, train-mode BN).

    One native training step; each layer is then re-run in fp32 PyTorch on the GPU path's
    OWN bf16 input and fed the GPU path's OWN upstream gradient, so bf16 ReLU-mask flips do
    not compound from layer to layer.  Inside a layer the reference rounds what the native
    path rounds -- the conv weights to bf16 (the kernels read bf16 copies of the fp32
    masters) and the pre-BN conv output to bf16 (stored bf16; the BN statistics and the
    ReLU mask come from the stored values) -- with straight-through gradients, so the ReLU
    masks agree and what is left is accumulation-order noise.  Every layer's output, input
    gradient and parameter gradients must match to a relative L2 error < 2e-2 (a 20 %
    gradient bug in any one layer fails it; the end-to-end test above only bounds the
    composed drift)."""
    _native_loaded()
    from featurenet_amd.models.featurenet3d import FeatureNet3D
    from featurenet_amd.ops import softmax_xent

    torch.manual_seed(11)
    m = FeatureNet3D().cuda().train()
    x = (torch.rand(32, 64, 64, 64, 1, device="cuda") < 0.3).to(torch.bfloat16)
    y = torch.randint(0, 24, (32,), device="cuda")
    layers = list(m.convs) + [m.fc1, m.fc2]
    rec = {}

    def hook(mod, inp, out):
        i = inp[0]
        if i.requires_grad:
            i.retain_grad()
        out.retain_grad()
        rec[mod] = (i, out)

    hs = [lay.register_forward_hook(hook) for lay in layers]
    bn_state = [(c.running_mean.clone(), c.running_var.clone()) for c in m.convs]
    logits = m(x)
    softmax_xent(logits, y).backward()
    for h in hs:
        h.remove()

    def rel(a, b):
        a, b = a.detach().float(), b.detach().float()
        return ((a - b).norm() / (b.norm() + 1e-12)).item()

    report = []
    for li, conv in enumerate(m.convs):
        xin, out = rec[conv]
        xr = xin.detach().float().requires_grad_(True)
        wr = conv.weight.detach().clone().requires_grad_(True)
        gr = conv.gamma.detach().clone().requires_grad_(True)
        br = conv.beta.detach().clone().requires_grad_(True)
        cs, ps = conv.specs(tuple(xin.shape))

        def bf16_st(t):                          # bf16 rounding, straight-through gradient
            return t + (t.to(torch.bfloat16).float() - t).detach()

        yr = bf16_st(ref.conv(xr, bf16_st(wr), None, cs))
        rm, rv = bn_state[li]
        zr = ref.batchnorm_act(yr, gr, br, rm.clone(), rv.clone(), True, conv.bn_momentum, conv.bn_eps, conv.act)
        if ps is not None:
            zr = ref.pool(zr, ps, conv.pool_kind)
        report.append((f"conv{li + 1}.out", rel(out, zr)))
        zr.backward(out.grad.float())
        report.append((f"conv{li + 1}.dW", rel(conv.weight.grad, wr.grad)))
        report.append((f"conv{li + 1}.dgamma", rel(conv.gamma.grad, gr.grad)))
        report.append((f"conv{li + 1}.dbeta", rel(conv.beta.grad, br.grad)))
        if li > 0:
            report.append((f"conv{li + 1}.dx", rel(xin.grad, xr.grad)))
    for name, lay in (("fc1", m.fc1), ("fc2", m.fc2)):
        xin, out = rec[lay]
        xr = xin.detach().float().reshape(xin.shape[0], -1).requires_grad_(True)
        wr = lay.weight.detach().clone().requires_grad_(True)
        br = lay.bias.detach().clone().requires_grad_(True)
        o = torch.nn.functional.linear(xr, wr, br)
        if name == "fc1":
            o = torch.relu(o)
        report.append((f"{name}.out", rel(out, o)))
        o.backward(out.grad.float())
        report.append((f"{name}.dW", rel(lay.weight.grad, wr.grad)))
        report.append((f"{name}.dx", rel(xin.grad.reshape(xr.shape), xr.grad)))
    print("\n".join(f"{n:16s} rel={r:.2e}" for n, r in report))
    bad = [(n, r) for n, r in report if not r < 2e-2]
    assert not bad, bad
