"""Block-scaled fp8 inference (OCP MX style): e4m3 activations with one E8M0 power-of-two scale per
(position, 32-channel block), applied inside ``v_mfma_scale_f32_16x16x128_f8f6f4`` as the halo
operand's scale (``conv_tile.hip`` BS instances), written by the producing epilogues.

Every check compares against an fp32 emulation of the same quantised operands: the block
quantiser against its definition (e = ceil(log2(amax / 448))), the scaled-MFMA conv against the
fp32 conv of the dequantised input and weights, the epilogue's block-scaled output against the
quantiser applied to the bf16 output.  (BASELINE.json config 5: 128^3 fp8 inference.)
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

from featurenet_amd import _native  # noqa: E402
from featurenet_amd.ops import reference as ref  # noqa: E402
from featurenet_amd.ops.spec import ConvSpec  # noqa: E402


def _spread(shape, lo=-8.0, hi=8.0, seed=0):
    """Activations whose magnitude varies by 2^16 across positions (one factor per position)."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(*shape, device="cuda", generator=g)
    f = torch.exp2(torch.rand(*shape[:-1], 1, device="cuda", generator=g) * (hi - lo) + lo)
    return (x * f).to(torch.bfloat16)


def test_block_quantiser_definition():
    from featurenet_amd.inference.fp8 import dequantize_fp8_block, quantize_fp8_block

    assert _native.kernels_available()
    x = _spread((4, 9, 10, 11, 64))
    x[0, 0, 0, 0] = 0                                   # an all-zero position
    q, sc = quantize_fp8_block(x)
    xf = x.float().reshape(-1, 2, 32)
    amax = xf.abs().amax(-1)
    e_ref = torch.ceil(torch.log2(amax / 448.0)).clamp(-127, 126)
    e_ref[amax == 0] = -127
    e = torch.stack([(sc.reshape(-1) >> (8 * j)) & 255 for j in range(2)], -1).float() - 127
    assert torch.equal(e, e_ref)
    d = dequantize_fp8_block(q, sc).reshape(-1, 2, 32)
    err = (d - xf).abs()
    # e4m3: 3 mantissa bits (half-ulp 2^-4 relative) down to the subnormal step 2^-9 x 2^e
    assert torch.all(err <= 0.0625 * xf.abs() + torch.exp2(e).unsqueeze(-1) * 2.0 ** -9)
    assert torch.all(d.abs() <= 448.0 * torch.exp2(e).unsqueeze(-1))


@pytest.mark.parametrize("cin,cout,k,dims,out_block", [
    (32, 32, 5, (3, 17, 16, 15), True),       # conv2-like: CS = 32, 4 taps per 128-k step, edge tiles
    (32, 64, 4, (2, 14, 13, 12), True),       # conv3-like
    (64, 64, 3, (2, 12, 13, 14), False),      # conv4-like: CS = 64, 2 taps per step, bf16 output
])
def test_block_scaled_conv_matches_emulation(cin, cout, k, dims, out_block):
    """The scaled-MFMA conv on block-scaled input vs the fp32 conv of the dequantised operands."""
    from featurenet_amd.inference.fp8 import Fp8Conv, dequantize_fp8_block, quantize_fp8_block
    from featurenet_amd.models.layers import Conv

    torch.manual_seed(4)
    conv = Conv(cin, cout, (k, k, k), 1, "valid", bias=True).cuda()
    with torch.no_grad():
        conv.bias.normal_(0, 0.1)
    x = _spread((*dims, cin), seed=1)
    xq, xs = quantize_fp8_block(x)
    layer = Fp8Conv(conv, 1.0, 1.0 if out_block else None, relu=True)
    spec = ConvSpec.make(x.shape, cout, (k, k, k))
    assert layer.tile_plan(spec, block=True) is not None, spec
    y, shape = layer((xq, xs), tuple(x.shape))
    yr = torch.relu(ref.conv(dequantize_fp8_block(xq, xs), layer.w_dequant, layer.bias, spec))
    if out_block:
        yq, ys = y
        assert yq.shape == tuple(shape) and ys.shape == tuple(shape[:-1])
        yd = dequantize_fp8_block(yq, ys)
        # e4m3 rounding of the output (3 mantissa bits) on top of the conv's accumulation order
        bound = 0.07 * yr.abs() + 1e-3 * yr.abs().amax(-1, keepdim=True)
        assert torch.all((yd - yr).abs() <= bound), ((yd - yr).abs() - bound).max()
    else:
        err = (y.float() - yr).abs().max().item()
        assert err <= 1e-2 * yr.abs().max().item(), err


def test_block_scales_keep_small_positions():
    """One position ~2^17 larger than the rest: per-tensor e4m3 pushes the others below e4m3's
    normal range (2^-6 of 448), the block-scaled path keeps them at e4m3 precision (the failure
    mode of a per-tensor scale)."""
    from featurenet_amd.inference.fp8 import Fp8Conv, dequantize_fp8_block, quantize_fp8_block
    from featurenet_amd.models.layers import Conv

    torch.manual_seed(5)
    conv = Conv(32, 32, (3, 3, 3), 1, "valid", bias=True).cuda()
    x = (torch.randn(2, 12, 12, 12, 32, device="cuda") * 0.01).to(torch.bfloat16)
    x[0, 0, 0, 0] = 2000.0                                # the outlier (sample 0 only)
    spec = ConvSpec.make(x.shape, 32, (3, 3, 3))
    xq, xs = quantize_fp8_block(x)
    lb = Fp8Conv(conv, 1.0, None, relu=False)
    yb, _ = lb((xq, xs), tuple(x.shape))
    ts = float(x.float().abs().amax()) / 448.0
    lt = Fp8Conv(conv, ts, None, relu=False)
    yt, _ = lt((x.float() / ts).to(torch.float8_e4m3fn).view(torch.uint8), tuple(x.shape))
    yr = ref.conv(x.float(), lb.w_dequant, lb.bias, spec)
    far = (slice(1, 2),)                                  # the second sample never sees the outlier
    eb = ((yb.float() - yr)[far].norm() / yr[far].norm()).item()
    et = ((yt.float() - yr)[far].norm() / yr[far].norm()).item()
    assert eb < 0.05 and eb * 4 < et, (eb, et)
    torch.testing.assert_close(dequantize_fp8_block(xq, xs)[1], x.float()[1], rtol=0.07, atol=1e-4)


def test_stem_block_output_equals_quantiser():
    """The bf16 stem's epilogue writing block-scaled e4m3 (Q8O BS instance) = the block quantiser
    applied to the stem's bf16 output, byte for byte."""
    from featurenet_amd.inference.fp8 import quantize_fp8_block
    from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig
    from featurenet_amd.ops import conv_tile
    from featurenet_amd.ops.conv import s2d_input, s2d_plan, s2d_weight

    torch.manual_seed(6)
    m = FeatureNet3D(FeatureNet3DConfig(input_size=48, num_classes=24)).cuda().eval()
    c1 = m.convs[0]
    x = (torch.rand(3, 48, 48, 48, 1, device="cuda") < 0.3).to(torch.bfloat16)
    spec = ConvSpec.make(tuple(x.shape), c1.cout, c1.kernel, c1.stride, c1.padding)
    f, spec2 = s2d_plan(spec)
    tp = conv_tile.fwd_plan(spec2)
    assert tp is not None and tp.CS == 8
    w2 = s2d_weight(c1.weight.detach().float(), f, spec, spec2)
    b = torch.randn(c1.cout, device="cuda") * 0.1
    x2 = s2d_input(x, f, spec2, (spec.pd, spec.ph, spec.pw))
    yq, ys = conv_tile.conv_fwd_q8_block(x2, w2, b, spec2, 1, tp)
    y, _ = conv_tile.conv_fwd(x2, w2, b, spec2, 1, False, tp)
    rq, rs = quantize_fp8_block(y)
    assert torch.equal(ys, rs)
    assert torch.equal(yq, rq)


def test_fp8_featurenet3d_block_matches_bf16():
    from featurenet_amd.inference.fp8 import quantize_model
    from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig

    torch.manual_seed(0)
    m = FeatureNet3D(FeatureNet3DConfig(input_size=64, num_classes=24)).cuda().eval()
    x = (torch.rand(6, 64, 64, 64, 1, device="cuda") < 0.3).to(torch.bfloat16)
    q = quantize_model(m, x[:4])
    assert q.block_mode(tuple(x.shape))
    with torch.no_grad():
        ref_logits = m(x).float()
        got = q(x).float()
    cos = torch.nn.functional.cosine_similarity(got.flatten(), ref_logits.flatten(), dim=0).item()
    assert cos > 0.98, cos


def test_quantize_fallback_reaches_the_agreement_bar():
    """quantize_model(fallback=True): the calibration check steps down (block scales -> per-tensor
    -> the bf16 model) until the fp8 model agrees with bf16 on >= FALLBACK_AT of the calibration
    set, and the model it returns agrees as much as it reports.  A random-init model (logits close
    together: a few % of fp8 noise flips the arg-max) exercises the steps; without fallback the
    same model keeps its block-scaled numerics and its (lower) agreement."""
    from featurenet_amd.inference import fp8 as F8
    from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig

    torch.manual_seed(3)
    m = FeatureNet3D(FeatureNet3DConfig(input_size=64, num_classes=24)).cuda().eval()
    x = (torch.rand(16, 64, 64, 64, 1, device="cuda") < 0.3).to(torch.bfloat16)
    import warnings

    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        q0 = F8.quantize_model(m, x, fp8_stem=False)
        q = F8.quantize_model(m, x, fp8_stem=False, fallback=True)
    assert q0.fallback is None and q0.calib_history[0][0] == "block"
    assert q.calib_history[0] == q0.calib_history[0]          # (same first step, same bits)
    assert q.calib_agreement >= F8.FALLBACK_AT or q.fallback == "bf16"
    if q0.calib_agreement >= F8.FALLBACK_AT:
        assert q.fallback is None
    else:
        assert q.fallback in ("per_tensor", "bf16") and len(q.calib_history) >= 2
    with torch.no_grad():
        a = m(x).float().argmax(-1)
        b = q(x).float().argmax(-1)
    assert round(float((a == b).float().mean()), 4) == q.calib_agreement


def test_trained_model_fp8_argmax_agreement():
    """FeatureNet-3D trained with the accuracy bench's recipe (procedural machining-feature voxels,
    64^3, 24 classes, 1,000 per class, 16 epochs, seed 0: ~20 s), then fp8 with the
    calibration-driven fallback: held-out top-1 agreement with the bf16 model >= 0.99 and top-1
    within 0.5 points (6 of 1,200 samples), on an fp8 path (not the bf16 fallback).  The step is
    bitwise repeatable, so the trained model is fixed by the tree's kernels: with the round-6
    32-column conv4 dgrad it was the seed-0 row of profiles/r6_fp8_fallback.md (block scales lose
    3.17 pt, the check moves it to per-tensor: 0.17 pt, 0.9983); with the 64-column dgrad's
    rounding the model differs and stays on block scales (calibration 0.9922; 0.50 pt, 0.9950)."""
    import numpy as np

    import featurenet_amd as fn
    from featurenet_amd.inference import fp8 as F8
    from featurenet_amd.training.data import unpack_voxels, voxel_dataset

    ds = voxel_dataset(1000 * 24, 50 * 24, size=64, num_classes=24, seed=0)
    res = fn.train("featurenet3d", data=ds, epochs=16, batch_size=128, lr=1e-3, seed=0, verbose=0, callbacks=[])
    model = res.model.eval()
    dev = next(model.parameters()).device

    def batch(xs, i, n):
        return unpack_voxels(torch.as_tensor(np.asarray(xs[i:i + n])).to(dev), 64).to(torch.bfloat16)

    q = F8.quantize_model(model, batch(ds.x_train, 0, 256), fallback=True)
    y = np.asarray(ds.y_test)
    pb, pq = [], []
    with torch.no_grad():
        for i in range(0, len(y), 128):
            xb = batch(ds.x_test, i, 128)
            pb.append(model(xb).float().argmax(-1).cpu())
            pq.append(q(xb).float().argmax(-1).cpu())
    pb, pq = torch.cat(pb).numpy(), torch.cat(pq).numpy()
    agree = float((pb == pq).mean())
    drop = float((pb == y).mean()) - float((pq == y).mean())
    print(f"bf16 top-1 {(pb == y).mean():.4f}, fp8 {q.calib_history}: agreement {agree:.4f}, drop {100 * drop:.2f} pt")
    assert float((pb == y).mean()) > 0.9                     # (a trained model)
    assert q.fallback != "bf16", q.calib_history
    assert agree >= 0.99, (agree, q.calib_history)
    assert drop <= 0.005 + 1e-9, (drop, q.calib_history)
    # the public API's fp8 path: the same quantisation from bit-packed calibration voxels
    labels, probs = fn.classify(model, ds.x_test, packed_size=64, fp8_calib=ds.x_train[:256])
    assert probs.shape == (len(y), 24)
    assert float((labels == pq).mean()) >= 0.995          # (batch 256 vs 128: the Dense split may differ)


def _e4m3(v: torch.Tensor) -> torch.Tensor:
    return v.to(torch.float8_e4m3fn).view(torch.uint8)


def _probe(a, b, sa, sb):
    d = torch.empty(64, 4, device="cuda")
    _native.kernels().mfma_scale_probe(a.data_ptr(), b.data_ptr(), sa.data_ptr(), sb.data_ptr(), d.data_ptr(),
                                       _native.stream(a))
    torch.cuda.synchronize()
    return d


def _emulate(a, b, sa, sb, kmap):
    """D[m][n] = sum_k A[m][k] B[k][n] 2^(sa(m, k/32) - 127) 2^(sb(n, k/32) - 127) with lane (r, g) byte
    i holding k = kmap(g, i) of row / column r, and the scale of (row r, block j) in lane r + 16 j."""
    av = a.view(torch.float8_e4m3fn).float().cpu()
    bv = b.view(torch.float8_e4m3fn).float().cpu()
    A = torch.zeros(16, 128)
    B = torch.zeros(128, 16)
    for lane in range(64):
        r, g = lane & 15, lane >> 4
        for i in range(32):
            k = kmap(g, i)
            A[r, k] = av[lane, i]
            B[k, r] = bv[lane, i]
    esa = (sa.cpu() & 255).float() - 127
    esb = (sb.cpu() & 255).float() - 127
    blk = torch.arange(128) // 32
    SA = torch.exp2(esa.view(4, 16).t()[:, blk])          # [m][k]: lane m + 16 * (k // 32)
    SB = torch.exp2(esb.view(4, 16).t()[:, blk])          # [n][k]
    D = (A * SA) @ (B * SB.t())
    out = torch.empty(64, 4)
    for lane in range(64):                                  # C layout: col = lane & 15, row = 4 (lane >> 4) + r
        for r in range(4):
            out[lane, r] = D[4 * (lane >> 4) + r, lane & 15]
    return out


KMAPS = {
    "contiguous": lambda g, i: 32 * g + i,                               # lane group g = k block g
    "split_halves": lambda g, i: 16 * g + i if i < 16 else 64 + 16 * g + (i - 16),
    "quads": lambda g, i: 8 * g + 32 * (i // 8) + i % 8,
}


def test_scaled_mfma_operand_layout():
    """One v_mfma_scale_f32_16x16x128_f8f6f4 with random e4m3 operands and random per-lane E8M0
    scales against an fp32 emulation: pins which K index each (lane, byte) holds and which lane's
    scale serves which 32-k block (the layout the block-scaled conv kernels are built on)."""
    torch.manual_seed(8)
    a = _e4m3(torch.randn(64, 32, device="cuda"))
    b = _e4m3(torch.randn(64, 32, device="cuda"))
    one = torch.full((64,), 127, dtype=torch.int32, device="cuda")
    d1 = _probe(a, b, one, one)
    sa = torch.randint(121, 134, (64,), dtype=torch.int32, device="cuda")
    sb = torch.randint(121, 134, (64,), dtype=torch.int32, device="cuda")
    d = _probe(a, b, sa, sb)
    res = {}
    for name, km in KMAPS.items():
        e1 = _emulate(a, b, one, one, km)
        e = _emulate(a, b, sa, sb, km)
        res[name] = ((d1.cpu() - e1).abs().max().item(), (d.cpu() - e).abs().max().item() / e.abs().max().item())
    print(res)
    assert res["contiguous"][0] < 1e-3 * d1.abs().max().item()          # the unscaled dot products
    # bytes 0-15 of lane group g are k = 16g.., bytes 16-31 are k = 64 + 16g..; block j's scale is
    # lane group j's (measured on MI355X; the block-scaled conv layout is built on this)
    assert res["split_halves"][1] < 1e-4, res
