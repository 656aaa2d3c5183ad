"""fp8 stem (``inference/fp8.py``): the ``s2d_tap_f8`` packing kernel against its torch
emulation, and the stem conv / whole model on the fp8 path against the bf16-stem fp8 path
and the bf16 model."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from featurenet_amd import _native  # noqa: E402
from featurenet_amd.inference import fp8 as F8  # noqa: E402
from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig  # noqa: E402


def _emulate(x, spec, inv_scale):
    N, D, H, W, _ = x.shape
    y = torch.zeros(N, spec.D, spec.H, spec.W, 32, device=x.device)
    w = torch.arange(spec.W, device=x.device)
    for j in range(4):
        for pd in range(2):
            for ph in range(2):
                for pw in range(2):
                    xd = 2 * torch.arange(spec.D, device=x.device) + pd
                    xh = 2 * torch.arange(spec.H, device=x.device) + ph
                    xw = 2 * (w + j) + pw
                    ok = (xd[:, None, None] < D) & (xh[None, :, None] < H) & (xw[None, None, :] < W)
                    v = x[:, xd.clamp(max=D - 1)][:, :, xh.clamp(max=H - 1)][:, :, :, xw.clamp(max=W - 1), 0].float()
                    y[..., 8 * j + pd * 4 + ph * 2 + pw] = torch.where(ok, v, torch.zeros_like(v))
    return (y * inv_scale).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)


def test_s2d_tap_f8_kernel_matches_emulation():
    assert _native.kernels_available()
    torch.manual_seed(0)
    x = (torch.randn(2, 40, 38, 44, 1, device="cuda") * 2).to(torch.bfloat16)

    class S:
        kernel, stride, padding, cout = (7, 7, 7), (2, 2, 2), "valid", 32
    spec = F8.stem_tap_plan(S, tuple(x.shape))
    assert spec is not None
    got = F8.stem_tap_input(x, spec, 0.05)
    ref = _emulate(x, spec, 1 / 0.05)
    assert got.shape == ref.shape
    same = (got == ref).float().mean().item()
    assert same > 0.9999, same


def test_fp8_stem_model_matches_bf16_stem_path():
    torch.manual_seed(0)
    m = FeatureNet3D(FeatureNet3DConfig(input_size=64, num_classes=24)).cuda().eval()
    x = (torch.rand(8, 64, 64, 64, 1, device="cuda") < 0.3).to(torch.bfloat16)
    q8 = F8.quantize_model(m, x[:4], fp8_stem=True)
    qb = F8.quantize_model(m, x[:4], fp8_stem=False)
    assert q8.stem is not None and F8.stem_tap_plan(m.convs[0], tuple(x.shape)) is not None
    with torch.no_grad():
        ref = m(x).float()
        a = q8(x).float()
        b = qb(x).float()
    cos_ab = torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()
    cos_ref = torch.nn.functional.cosine_similarity(a.flatten(), ref.flatten(), dim=0).item()
    assert cos_ab > 0.99 and cos_ref > 0.97, (cos_ab, cos_ref)


@pytest.mark.parametrize("N,S,C,K", [(2, 22, 64, 64), (3, 14, 32, 32), (2, 54, 64, 64)])
def test_fp8_fused_pool_matches_unfused(N, S, C, K):
    """conv_tile F8 with the fused 2^3 max-pool epilogue == the plain F8 kernel (bf16 output)
    followed by relu + max-pool in torch (identical conv arithmetic; bf16 rounding of the max)."""
    from featurenet_amd.ops import conv_tile as ct
    from featurenet_amd.ops.spec import ConvSpec

    torch.manual_seed(1)
    xq = (torch.randn(N, S, S, S, C, device="cuda") * 8).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    wq = (torch.randn(K, 27, C, device="cuda") * 16).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    spec = ConvSpec.make((N, S, S, S, C), K, 3, 1, "valid")
    scale = torch.rand(K, device="cuda") * 1e-3 + 1e-4
    bias = torch.randn(K, device="cuda") * 0.1
    p0 = ct.plan(N, (spec.OD, spec.OH, spec.OW), (3, 3, 3), C, K, f8=True)
    pp = ct.plan(N, (spec.OD, spec.OH, spec.OW), (3, 3, 3), C, K, f8=True, pool=True)
    assert p0 is not None and pp is not None and pp.pool
    y = ct.conv_fwd_f8(xq, ct.pack_weights_f8(wq, p0), scale, bias, spec, p0, True, None)
    ref = torch.nn.functional.max_pool3d(y.float().permute(0, 4, 1, 2, 3), 2).permute(0, 2, 3, 4, 1)
    got = ct.conv_fwd_f8(xq, ct.pack_weights_f8(wq, pp), scale, bias, spec, pp, True, None)
    assert got.shape == ref.shape
    torch.testing.assert_close(got.float(), ref, rtol=1e-2, atol=1e-3)


def test_tile_f8_matches_halo_f8_model(monkeypatch):
    """Same quantised model through the fp8 tile kernel and the fp8 halo kernel (bf16 stem,
    unfused pool in both): identical fp8 products, fp32 accumulation in a different order --
    the logits agree to ~1e-2 relative and the intermediate fp8 activations almost exactly.
    Per-tensor activation scales in both (the halo kernel has no block-scaled form; the block
    path is checked against its own emulation in test_fp8_block_gpu.py)."""
    torch.manual_seed(3)
    m = FeatureNet3D(FeatureNet3DConfig(input_size=64, num_classes=24)).cuda().eval()
    x = (torch.rand(8, 64, 64, 64, 1, device="cuda") < 0.3).to(torch.bfloat16)
    q = F8.quantize_model(m, x[:4], fp8_stem=False)
    monkeypatch.setenv("FN_F8_POOL", "0")
    monkeypatch.setenv("FN_F8_BLOCK", "0")
    outs = {}
    for tile in ("1", "0"):
        monkeypatch.setenv("FN_F8_TILE", tile)
        acts = []
        with torch.no_grad():
            c1 = m.convs[0]
            from featurenet_amd import ops
            from featurenet_amd.ops.spec import ConvSpec
            spec = ConvSpec.make(tuple(x.shape), c1.cout, c1.kernel, c1.stride, c1.padding)
            xq = F8.quantize_fp8_act(ops.conv(x, q.c1_w, q.c1_b, spec, "relu"), q.act_scales[0])
            shape = spec.out_shape5
            for layer in q.layers:
                xq, shape = layer(xq, shape)
                acts.append(xq)
            outs[tile] = (acts, q(x).float())
    for a, b in zip(outs["1"][0][:-1], outs["0"][0][:-1]):          # fp8 intermediate activations
        same = (a == b).float().mean().item()
        assert same > 0.995, same
    a, b = outs["1"][0][-1].float(), outs["0"][0][-1].float()        # conv4 (bf16 out)
    assert ((a - b).norm() / b.norm()).item() < 2e-2
    la, lb = outs["1"][1], outs["0"][1]
    assert ((la - lb).norm() / lb.norm()).item() < 2e-2


def test_bf16_stem_e4m3_epilogue_matches_quant_pass(monkeypatch):
    """The default fp8 model's bf16 stem writes e4m3 from the tile epilogue: same bytes as the
    bf16 stem output followed by the quantisation pass (FN_F8_STEM_Q8=0)."""
    torch.manual_seed(4)
    m = FeatureNet3D(FeatureNet3DConfig(input_size=64, num_classes=24)).cuda().eval()
    x = (torch.rand(4, 64, 64, 64, 1, device="cuda") < 0.3).to(torch.bfloat16)
    q = F8.quantize_model(m, x)
    assert q.stem is None
    from featurenet_amd.ops.spec import ConvSpec
    c1 = m.convs[0]
    spec = ConvSpec.make(tuple(x.shape), c1.cout, c1.kernel, c1.stride, c1.padding)
    with torch.no_grad():
        a = q._bf16_stem_fp8_out(x, spec)
        from featurenet_amd import ops
        b = F8.quantize_fp8_act(ops.conv(x, q.c1_w, q.c1_b, spec, "relu"), q.act_scales[0])
    assert a is not None and a.shape == b.shape and a.dtype == torch.uint8
    same = (a == b).float().mean().item()
    assert same > 0.999, same


@pytest.mark.skipif(not __import__("featurenet_amd.ops.conv_tile", fromlist=["x"]).experiments_built(),
                    reason="the int8 stem instance is an experiment build (FN_BUILD_EXPERIMENTS=1)")
def test_int8_tile_kernel_exact():
    """The int8 instance of the fp8 tile kernel (two v_mfma_i32_16x16x64_i8 per fragment pair)
    against an exact integer conv: int8 x, int8 w, int32 sums, then scale + bias + relu."""
    from featurenet_amd.ops import conv_tile as ct
    from featurenet_amd.ops.spec import ConvSpec

    torch.manual_seed(7)
    N, S, C, K = 2, 12, 32, 32
    xi = torch.randint(-20, 21, (N, S, S, S, C), device="cuda", dtype=torch.int8)
    wi = torch.randint(-127, 128, (K, 4, 4, 1, C), device="cuda", dtype=torch.int8)
    spec = ConvSpec.make((N, S, S, S, C), K, (4, 4, 1), 1, "valid")
    p = ct.plan(N, (spec.OD, spec.OH, spec.OW), (4, 4, 1), C, K, f8=True)
    assert p is not None
    scale = torch.rand(K, device="cuda") * 1e-3 + 1e-4
    bias = torch.randn(K, device="cuda") * 0.1
    wpk = ct.pack_weights_f8(wi.view(torch.uint8).reshape(K, 16, C), p)
    y = ct.conv_fwd_f8(xi.view(torch.uint8), wpk, scale, bias, spec, p, True, None, i8=True)
    acc = torch.nn.functional.conv3d(xi.double().permute(0, 4, 1, 2, 3), wi.double().permute(0, 4, 1, 2, 3))
    ref = torch.relu(acc.permute(0, 2, 3, 4, 1) * scale.double() + bias.double())
    torch.testing.assert_close(y.double(), ref, rtol=8e-3, atol=1e-3)   # (bf16 output rounding)


@pytest.mark.skipif(not __import__("featurenet_amd.ops.conv_tile", fromlist=["x"]).experiments_built(),
                    reason="the int8 stem instance is an experiment build (FN_BUILD_EXPERIMENTS=1)")
def test_int8_stem_model_matches_bf16_model():
    """The fp8 model with the int8 stem (FN_F8_STEM=i8): closer to the bf16 model than the e4m3
    stem, as close as the bf16 stem."""
    torch.manual_seed(0)
    m = FeatureNet3D(FeatureNet3DConfig(input_size=64, num_classes=24)).cuda().eval()
    x = (torch.rand(8, 64, 64, 64, 1, device="cuda") < 0.3).to(torch.bfloat16)
    qi = F8.quantize_model(m, x[:4], fp8_stem="i8")
    qb = F8.quantize_model(m, x[:4], fp8_stem="bf16")
    assert qi.stem is not None and qi.stem.int8
    with torch.no_grad():
        ref = m(x).float()
        a = qi(x).float()
        b = qb(x).float()
    cos = lambda u, v: torch.nn.functional.cosine_similarity(u.flatten(), v.flatten(), dim=0).item()  # noqa: E731
    assert cos(a, b) > 0.995 and cos(a, ref) >= cos(b, ref) - 0.01, (cos(a, b), cos(a, ref), cos(b, ref))
