"""BN + activation of a conv's input inside the conv_tile forward's loader (``conv_tile.hip``
``xform_job``, ``ops/bnfuse.py`` defer / settle) against the separate ``bn_apply`` pass.

The loader applies the same fma, activation and bf16 rounding as ``bn_apply_kernel``, so the
conv output, its BN-statistics slab, the z it writes back for the positions its tiles own and the
relu-mask bytes must all be bit-identical to bn_apply followed by the plain conv -- at the
FeatureNet-3D layer shapes (valid convs: every halo interior), same-padded shapes (border tiles:
the zero page's padding must stay zero, not act(shift)), several slices per tile and several
column blocks.  At model level the training step with the prologue gives the same loss and
gradients bit for bit as with ``FN_BN_PROLOGUE=0``.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

from featurenet_amd import _native  # noqa: E402
from featurenet_amd.ops import conv_tile as ct  # noqa: E402
from featurenet_amd.ops.spec import ConvSpec  # noqa: E402

CASES = [
    # (N, D, H, W, C, K, kernel, padding, act)
    (2, 29, 29, 29, 32, 32, (5, 5, 5), "valid", 1),   # FeatureNet-3D conv2 (input: the stem's BN + ReLU)
    (2, 25, 25, 25, 32, 64, (4, 4, 4), "valid", 1),   # conv3
    (3, 22, 22, 22, 64, 64, (3, 3, 3), "valid", 1),   # conv4: 2 slices per tile, 2 column blocks
    (3, 11, 12, 13, 16, 48, (3, 3, 3), "same", 1),    # border tiles: zero-page padding positions
    (2, 9, 10, 11, 64, 64, (3, 3, 3), "same", 1),     # 64 input channels: CS 32/64
    (3, 10, 11, 12, 8, 16, (3, 3, 3), "same", 1),     # 8-channel slices
]


@pytest.mark.parametrize("case", CASES)
def test_prologue_matches_bn_apply(case):
    assert _native.kernels_available(), "HIP kernel library (_C) must be built and loadable on the GPU box"
    N, D, H, W, C, K, k, pad, act = case
    torch.manual_seed(0)
    dev = "cuda"
    y = torch.randn(N, D, H, W, C, device=dev).to(torch.bfloat16)
    mean = torch.randn(C, device=dev) * 0.2
    invstd = torch.rand(C, device=dev) + 0.5
    scale = torch.randn(C, device=dev)
    shift = torch.randn(C, device=dev) * 0.5
    prm = torch.stack([mean, invstd, scale, shift]).contiguous()
    Kn = _native.kernels()
    st = _native.stream(y)
    z_ref = torch.empty_like(y)
    m_ref = torch.empty(y.numel() // 8, dtype=torch.uint8, device=dev)
    Kn.bn_apply(y.data_ptr(), prm[2].data_ptr(), prm[3].data_ptr(), z_ref.data_ptr(), y.numel(), C, act, st,
                m_ref.data_ptr(), m_ref.numel())
    spec = ConvSpec.make(y.shape, K, k, 1, pad)
    w = (torch.randn(K, spec.KD, spec.KH, spec.KW, C, device=dev) * 0.05).to(torch.bfloat16).float()
    p = ct.fwd_plan(spec)
    assert p is not None
    o_ref, s_ref = ct.conv_fwd(z_ref, w, None, spec, 0, True, p)
    # poison z and the mask: every position must be written by exactly the tile that owns it
    z = torch.full_like(y, float("nan"))
    m = torch.full_like(m_ref, 0xA5)
    o, s = ct.conv_fwd(z, w, None, spec, 0, True, p, pro=(y, prm, act, z, m))
    torch.cuda.synchronize()
    assert torch.equal(z.view(torch.int16), z_ref.view(torch.int16))
    if act == 1:
        assert torch.equal(m, m_ref)
    assert torch.equal(o, o_ref)
    assert torch.equal(s, s_ref)


@pytest.mark.parametrize("nw", ["8", "4"])
@pytest.mark.parametrize("case", CASES)
def test_wgrad_prologue_matches_bn_apply(case, nw, monkeypatch):
    """conv_wtile with the prologue (x = y, normalised in LDS by whoever DMA'd the slots: each wave
    in the loaderless form, the loader wave in the 4-wave form) against the weight gradient of the
    bn_apply output, bit for bit."""
    from featurenet_amd.ops import conv_wtile as cw

    N, D, H, W, C, K, k, pad, act = case
    monkeypatch.setenv("FN_WTILE_NW", nw)
    monkeypatch.setattr(cw, "_PLANS", {})
    torch.manual_seed(2)
    dev = "cuda"
    y = torch.randn(N, D, H, W, C, device=dev).to(torch.bfloat16)
    prm = torch.stack([torch.zeros(C, device=dev), torch.ones(C, device=dev), torch.randn(C, device=dev),
                       torch.randn(C, device=dev) * 0.5]).contiguous()
    Kn = _native.kernels()
    z_ref = torch.empty_like(y)
    Kn.bn_apply(y.data_ptr(), prm[2].data_ptr(), prm[3].data_ptr(), z_ref.data_ptr(), y.numel(), C, act,
                _native.stream(y), 0, 0)
    spec = ConvSpec.make(y.shape, K, k, 1, pad)
    if not _native.kernels().conv_wtile_prologue_built():
        pytest.skip("conv_wtile's x-halo prologue is in experiment builds only (FN_BUILD_EXPERIMENTS=1)")
    p = cw.plan(spec)
    if p is None or not cw.prologue_ok(p):
        pytest.skip("no conv_wtile plan with the prologue form for this shape")
    dy = torch.randn(spec.out_shape5, device=dev).to(torch.bfloat16)
    dw_ref = cw.conv_wgrad(dy, z_ref, spec, p).clone()
    dw = cw.conv_wgrad(dy, y, spec, p, pro=(prm, act))
    torch.cuda.synchronize()
    assert torch.equal(dw, dw_ref), float((dw - dw_ref).norm() / dw_ref.norm())


def test_prologue_without_mask_or_z_writeback():
    """pz / pmask are optional: the conv output alone from y."""
    torch.manual_seed(1)
    dev = "cuda"
    y = torch.randn(2, 25, 25, 25, 32, device=dev).to(torch.bfloat16)
    prm = torch.stack([torch.zeros(32, device=dev), torch.ones(32, device=dev), torch.rand(32, device=dev) + 0.5,
                       torch.randn(32, device=dev) * 0.3]).contiguous()
    z_ref = torch.relu(y.float() * prm[2] + prm[3]).to(torch.bfloat16)
    spec = ConvSpec.make(y.shape, 64, (4, 4, 4), 1, "valid")
    w = (torch.randn(64, 4, 4, 4, 32, device=dev) * 0.05).to(torch.bfloat16).float()
    p = ct.fwd_plan(spec)
    o_ref, _ = ct.conv_fwd(z_ref, w, None, spec, 0, False, p)
    z = torch.empty_like(y)
    geom_ok = ct.conv_fwd(z, w, None, spec, 0, False, p, pro=(y, prm, 1, z, None))
    torch.cuda.synchronize()
    # (fp32 torch z with one rounding: the same bits as the kernel's fma + bf16 rounding except in
    # rare double-rounding cases -- compare the conv outputs loosely)
    rel = ((geom_ok[0].float() - o_ref.float()).norm() / o_ref.float().norm()).item()
    assert rel < 1e-2, rel


def _step(monkeypatch, prologue: str, wgrad: str = "0"):
    from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig
    from featurenet_amd.ops import softmax_xent
    from featurenet_amd.training.flat import FlatParams

    monkeypatch.setenv("FN_BN_PROLOGUE", prologue)
    monkeypatch.setenv("FN_BN_PROLOGUE_WGRAD", wgrad)
    torch.manual_seed(5)
    dev = torch.device("cuda", 0)
    model = FeatureNet3D(FeatureNet3DConfig()).to(dev)
    flat = FlatParams(model)
    g = torch.Generator().manual_seed(9)
    x = (torch.rand(4, 64, 64, 64, 1, generator=g) < 0.3).to(torch.uint8).to(dev)
    yl = torch.randint(0, 24, (4,), generator=g).to(dev)
    flat.zero_grad()
    loss = softmax_xent(model(x), yl)
    loss.backward()
    torch.cuda.synchronize()
    return loss.detach().clone(), flat.grad.clone(), [b.clone() for b in model.buffers()]


@pytest.mark.parametrize("wgrad", ["0", "1"])
def test_model_step_prologue_bitwise(monkeypatch, wgrad):
    """The FeatureNet-3D step with the prologue (z written by the forward's loader, or -- wgrad
    "1" -- never written, the weight gradients normalising y themselves) against bn_apply."""
    l0, g0, b0 = _step(monkeypatch, "0")
    l1, g1, b1 = _step(monkeypatch, "1", wgrad)
    assert torch.equal(l0, l1)
    assert torch.equal(g0, g1), float((g0 - g1).norm() / g0.norm())
    assert all(torch.equal(a, b) for a, b in zip(b0, b1))   # running statistics
