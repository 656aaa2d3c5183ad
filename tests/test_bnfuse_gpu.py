"""BN-backward statistics fused into the consuming conv's dgrad (ops/bnfuse.py: the relu-mask
epilogue and the statistics identity, the max-pool backward's moments): the fused paths must give
the same parameter and input gradients as the separate colstats pass, and must actually take the
fused branch."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from featurenet_amd import _native  # noqa: E402
from featurenet_amd.ops import bn as bnmod  # noqa: E402
from featurenet_amd.ops import bnfuse  # noqa: E402


def _grads(model, x, fuse: bool, monkeypatch):
    monkeypatch.setenv("FN_POOL_BN_STATS", "1" if fuse else "0")
    model.zero_grad(set_to_none=True)
    out = model(x)
    loss = (out.float() * torch.linspace(-1, 1, out.shape[-1], device=x.device)).sum()
    loss.backward()
    return {n: p.grad.detach().float().clone() for n, p in model.named_parameters()}


def _count_fused(monkeypatch):
    calls = {"fused": 0}
    orig = bnfuse.take

    def take(dz, y):
        r = orig(dz, y)
        calls["fused"] += r is not None
        return r

    monkeypatch.setattr(bnmod.bnfuse, "take", take)
    return calls


@pytest.mark.parametrize("N,S,C", [(2, 20, 64), (4, 10, 32), (3, 8, 16)])
def test_pool_bwd_bn_stats_match_colstats(monkeypatch, N, S, C):
    """Max-pool backward with the BN-backward moments (pool_bwd_stats) vs pool_bwd + colstats."""
    from featurenet_amd.models.layers import Conv

    torch.manual_seed(2)
    dev = torch.device("cuda", 0)
    layer = Conv(C, C, 3, 1, "same", bn=True, act="relu", pool=(2, 2, 2), init="he").to(dev)
    x = torch.randn(N, S, S, S, C, device=dev).to(torch.bfloat16)
    g0 = _grads(layer, x, False, monkeypatch)
    g1 = _grads(layer, x, True, monkeypatch)
    for n in g0:
        a, b = g0[n], g1[n]
        err = (a - b).abs().max().item() / max(a.abs().max().item(), 1e-6)
        assert err < 2e-3, f"{n}: rel err {err:.2e}"


@pytest.mark.parametrize("N,S,C", [(2, 20, 64), (3, 8, 16), (4, 6, 8)])
def test_pool_bn_bwd_apply_matches_separate_passes(monkeypatch, N, S, C):
    """BN+ReLU+max-pool backward in one pass (pool_bn_bwd_apply: no sparse dz tensor) vs
    pool_bwd + bn_bwd_apply: same input and parameter gradients."""
    from featurenet_amd.models.layers import Conv

    torch.manual_seed(3)
    dev = torch.device("cuda", 0)
    layer = Conv(C, C, 3, 1, "same", bn=True, act="relu", pool=(2, 2, 2), init="he").to(dev)
    x0 = torch.randn(N, S, S, S, C, device=dev).to(torch.bfloat16)
    Kn = _native.kernels()
    calls = {"n": 0}
    orig = Kn.pool_bn_bwd_apply

    def counted(*a, **k):
        calls["n"] += 1
        return orig(*a, **k)

    monkeypatch.setattr(Kn, "pool_bn_bwd_apply", counted)
    res = {}
    for apply in ("0", "1"):
        monkeypatch.setenv("FN_POOL_BN_APPLY", apply)
        x = x0.clone().requires_grad_(True)
        g = _grads(layer, x, True, monkeypatch)
        g["x"] = x.grad.detach().float().clone()
        res[apply] = g
    for n in res["0"]:
        a, b = res["0"][n], res["1"][n]
        err = (a - b).abs().max().item() / max(a.abs().max().item(), 1e-6)
        assert err < 2e-3, f"{n}: rel err {err:.2e}"
    assert calls["n"] == 1


@pytest.mark.parametrize("S", [16, 32])
def test_seg_head_bn_in_pointwise_matches_unfused(monkeypatch, S):
    """FeatureNet3DSeg training step with the decoder BN + ReLU inside the 1x1 head's pointwise
    kernels (BatchNormActPointwiseFn) vs bn_apply + plain head: same logits and gradients."""
    from featurenet_amd.models.featurenet3d import FeatureNet3DSeg
    from featurenet_amd.ops import softmax_xent

    torch.manual_seed(3)
    dev = torch.device("cuda", 0)
    model = FeatureNet3DSeg(input_size=S).to(dev).train()
    x = (torch.rand(2, S, S, S, 1, device=dev) < 0.3).to(torch.bfloat16)
    lab = torch.randint(0, 25, (2, S, S, S), device=dev)
    res = []
    monkeypatch.setenv("FN_SUBPIXEL", "0")      # this pair isolates the BN-in-pointwise fusion
    for fuse in ("0", "0", "1"):                 # (the sub-pixel decoder: tests/test_subpixel_gpu.py)
        monkeypatch.setenv("FN_BN_PW_FUSE", fuse)
        model.zero_grad(set_to_none=True)
        out = model(x)
        softmax_xent(out, lab).backward()
        res.append((out.detach().float(), {n: p.grad.detach().float().clone() for n, p in model.named_parameters()}))
    (o0, g0), (o0b, g0b), (o1, g1) = res
    # the unfused path against itself: bitwise (deterministic kernels, tests/test_determinism_gpu.py)
    assert torch.equal(o0, o0b) and all(torch.equal(g0[n], g0b[n]) for n in g0)
    assert (o0 - o1).abs().max().item() <= 5e-3 * o0.abs().max().item()
    errs = {n: (g0[n] - g1[n]).abs().max().item() / max(g0[n].abs().max().item(), 1e-6) for n in g0}
    print({n: f"{e:.2e}" for n, e in errs.items()})
    for n, err in errs.items():
        assert err < 5e-3, f"{n}: rel err {err:.2e}"


def test_forked_bn_output_falls_back(monkeypatch):
    """A BN output with two consumers (a conv and an identity branch): autograd adds the
    identity branch's gradient into the conv's dx, so the dgrad-epilogue slab of the statistics
    identity (conv branch only) must not be used -- the gradients must equal the colstats path."""
    from torch import nn

    from featurenet_amd.models.layers import Conv

    class Fork(nn.Module):
        def __init__(self):
            super().__init__()
            self.a = Conv(32, 32, 3, 1, "valid", bn=True, act="relu", init="he")
            self.b = Conv(32, 32, 3, 1, "same", bn=False, act=None, init="he")

        def forward(self, x):
            z = self.a(x)
            return self.b(z) + z                # two consumers of the BN+ReLU output

    monkeypatch.setenv("FN_CONV_TILE", "2")
    torch.manual_seed(3)
    dev = torch.device("cuda", 0)
    model = Fork().to(dev)
    x = torch.randn(2, 18, 18, 18, 32, device=dev).to(torch.bfloat16)
    g0 = _grads_ident(model, x, False, monkeypatch)
    g1 = _grads_ident(model, x, True, monkeypatch)
    for n in g0:
        a, b = g0[n], g1[n]
        err = (a - b).abs().max().item() / max(a.abs().max().item(), 1e-6)
        assert err < 2e-3, f"{n}: rel err {err:.2e}"


def _count_identity(monkeypatch):
    from featurenet_amd.ops import bn as bnm

    calls = {"identity": 0}
    orig = bnm._bwd_identity

    def wrapped(*a, **k):
        calls["identity"] += 1
        return orig(*a, **k)

    monkeypatch.setattr(bnm, "_bwd_identity", wrapped)
    return calls


def _grads_ident(model, x, on: bool, monkeypatch):
    monkeypatch.setenv("FN_BN_IDENTITY", "1" if on else "0")
    model.zero_grad(set_to_none=True)
    out = model(x)
    loss = (out.float() * torch.linspace(-1, 1, out.shape[-1], device=x.device)).sum()
    loss.backward()
    return {n: p.grad.detach().float().clone() for n, p in model.named_parameters()}


def test_identity_featurenet3d_matches_colstats(monkeypatch):
    """Production shapes (64^3, batch 8): the BN backward of conv1-3's BNs from the statistics
    identity (relu mask in the dgrad epilogue, S = sum W . dW) against the colstats pass."""
    from featurenet_amd.models.featurenet3d import FeatureNet3D

    torch.manual_seed(2)
    dev = torch.device("cuda", 0)
    model = FeatureNet3D().to(dev)
    x = (torch.rand(8, 64, 64, 64, 1, device=dev) < 0.3).to(torch.bfloat16)
    calls = _count_identity(monkeypatch)
    g0 = _grads_ident(model, x, False, monkeypatch)
    assert calls["identity"] == 0
    g1 = _grads_ident(model, x, True, monkeypatch)
    assert calls["identity"] == 3, f"identity path taken {calls['identity']} times (conv2-4 inputs)"
    g2 = _grads_ident(model, x, False, monkeypatch)
    # off vs off: the same bits (static tile schedules and fixed-order partial sums make the step
    # repeatable; before them the BN statistics' summation order followed the dynamic tile
    # schedule and the first step in a process differed from later ones).  Identity vs colstats:
    # relative L2 -- the two BN backwards round differently in bf16 (the identity pieces are checked
    # exactly in test_identity_pieces_exact)
    for n in g0:
        assert torch.equal(g0[n], g2[n]), f"{n}: off / off not bitwise equal"
    rl2 = lambda u, v: ((u - v).norm() / u.norm().clamp_min(1e-12)).item()  # noqa: E731
    errs = {n: rl2(g0[n], g1[n]) for n in g0}
    print({n: f"{e:.2e}" for n, e in errs.items()})
    for n, e in errs.items():
        assert e < 1e-2, f"{n}: rel L2 err {e:.2e}"


@pytest.mark.parametrize("gscale", [1.0, -0.5, 1e-4])
def test_identity_any_gamma(monkeypatch, gscale):
    """conv -> BN(relu) -> conv with gamma positive, negative or ~0 and large beta: the identity
    path's gradients equal the colstats path's (no division by gamma anywhere)."""
    from torch import nn

    from featurenet_amd.models.layers import Conv

    monkeypatch.setenv("FN_CONV_TILE", "2")
    torch.manual_seed(3)
    dev = torch.device("cuda", 0)
    model = nn.Sequential(Conv(16, 32, 3, 1, "valid", bn=True, act="relu", init="he"),
                          Conv(32, 32, 3, 1, "valid", bn=True, act="relu", init="he")).to(dev)
    with torch.no_grad():
        for m in model.modules():
            if getattr(m, "gamma", None) is not None:
                m.gamma.mul_(gscale)
                m.beta.add_(torch.linspace(-2, 3, m.beta.numel(), device=dev))
    x = torch.randn(4, 20, 20, 20, 16, device=dev).to(torch.bfloat16)
    calls = _count_identity(monkeypatch)
    g0 = _grads_ident(model, x, False, monkeypatch)
    g1 = _grads_ident(model, x, True, monkeypatch)
    g2 = _grads_ident(model, x, False, monkeypatch)
    assert calls["identity"] >= 1
    # (gamma 1e-4: the gradients below the second BN are ~1e-4 of their usual scale, where the
    # two BN backwards' different bf16 roundings are largest; a division by gamma would be off by
    # orders of magnitude.  The off/off spread is zero since the step is bit-repeatable: the bound
    # is 1e-2, the 4x-spread term kept for boxes where it is not)
    rel = lambda u, v: (u - v).abs().max().item() / max(u.abs().max().item(), 1e-6)  # noqa: E731
    for n in g0:
        err, err0 = rel(g0[n], g1[n]), rel(g0[n], g2[n])
        assert err < max(1e-2, 4 * err0), f"{n}: rel err {err:.2e} (off/off {err0:.2e})"


@pytest.mark.parametrize("N,S,C,K,k", [(8, 22, 64, 64, 3), (4, 29, 32, 32, 5), (4, 25, 32, 64, 4)])
def test_identity_pieces_exact(N, S, C, K, k):
    """The statistics identity's pieces on one conv (FeatureNet-3D conv2-4 shapes): the masked
    dgrad stores dz unchanged and the column sums of dz * relu'(z), the conv's weight gradient is
    unchanged by it, bn_wdot equals torch's sum bf16(W) * dW, and that sum equals sum dz * z."""
    import importlib

    from featurenet_amd.ops import conv_tile as ct
    from featurenet_amd.ops.spec import ConvSpec

    cv = importlib.import_module("featurenet_amd.ops.conv")
    torch.manual_seed(0)
    x = torch.relu(torch.randn(N, S, S, S, C, device="cuda")).to(torch.bfloat16)
    spec = ConvSpec.make(x.shape, K, k, 1, "valid")
    w = torch.randn(K, k, k, k, C, device="cuda") * 0.05
    dy = torch.randn(spec.out_shape5, device="cuda").to(torch.bfloat16)
    bits = (x.reshape(-1, 8) > 0).to(torch.uint8)
    mask = (bits * (2 ** torch.arange(8, device="cuda", dtype=torch.uint8))).sum(-1).to(torch.uint8).contiguous()
    p = ct.dgrad_plan(spec)
    assert p is not None and ct.mask_dgrad_ok(p, C)
    dz = ct.conv_dgrad(dy, w, spec, p)
    dw0 = cv.native_conv_wgrad(dy, x, spec).clone()
    g, ident = ct.conv_dgrad(dy, w, spec, p, bn=(x, None, 1, mask))
    assert isinstance(ident, tuple) and ident[0] == "identity"
    dw1 = cv.native_conv_wgrad(dy, x, spec).clone()
    ref = dz.float() * (x.float() > 0)
    assert torch.equal(g, dz)                    # dx stored whole (the true gradient of z)
    sg = ident[1][:, 0].sum(0)
    rs = ref.reshape(-1, C).sum(0)
    assert ((sg - rs).abs().max() / rs.abs().max()).item() < 1e-5
    assert torch.equal(dw0, dw1)
    S_k = cv.bn_wdot(w, dw0, spec).sum(0)
    S_t = (w.to(torch.bfloat16).float() * dw0).reshape(-1, C).sum(0)
    S_z = (dz.float() * x.float()).reshape(-1, C).sum(0)
    assert ((S_k - S_t).abs().max() / S_t.abs().max()).item() < 1e-5
    assert ((S_k - S_z).abs().max() / S_z.abs().max()).item() < 5e-3   # (dz rounded to bf16 here)
