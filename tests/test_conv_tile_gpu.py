"""Big-tile conv kernel (``csrc/kernels/conv_tile.hip`` on v_mfma_f32_16x16x32_bf16) vs the fp32
PyTorch reference.

Forward (bias + activation epilogue, BN statistics epilogue) and dgrad at the
FeatureNet-3D layer shapes, at a small batch and at a production-size batch
whose tile count is many times the 256 persistent workgroups (the chunked tile schedule
with BN statistics, the per-tile one without, halo double buffering across jobs, multi-slice
jobs), plus
same-padded / 2-D / multi-column-block shapes from the NAS search space.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

from featurenet_amd import _native  # noqa: E402
from featurenet_amd.ops import conv_tile as ct  # noqa: E402
from featurenet_amd.ops import reference as ref  # noqa: E402
from featurenet_amd.ops.spec import ConvSpec  # noqa: E402


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item(), (a - b).abs().max().item() / (b.abs().max().item() + 1e-12)


CASES = [
    # (N, D, H, W, C, K, kernel, padding)
    (2, 29, 29, 29, 32, 32, (5, 5, 5), "valid"),     # FeatureNet-3D conv2
    (2, 25, 25, 25, 32, 64, (4, 4, 4), "valid"),     # conv3
    (2, 22, 22, 22, 64, 64, (3, 3, 3), "valid"),     # conv4
    (16, 29, 29, 29, 32, 32, (5, 5, 5), "valid"),    # conv2, 400 tiles > 256 workgroups
    (24, 22, 22, 22, 64, 64, (3, 3, 3), "valid"),    # conv4, 2 slices per tile, 384 tiles
    (3, 11, 12, 13, 16, 48, (3, 3, 3), "same"),      # same padding, 48 columns (16x16 kernel only)
    (2, 9, 10, 11, 32, 96, (3, 3, 3), "same"),       # 2 column blocks
    (2, 9, 10, 11, 32, 128, (3, 3, 3), "same"),      # 4 column blocks of 32
    (4, 29, 29, 29, 32, 32, (5, 5, 5), "valid"),     # conv2, CS = 16 plans
    (2, 9, 10, 11, 64, 64, (3, 3, 3), "same"),       # 64 input channels: CS = 64 / 32 slices
    (4, 1, 40, 37, 32, 32, (1, 5, 5), "same"),       # 2-D conv
    (6, 32, 32, 32, 8, 32, (4, 4, 4), "valid"),      # FeatureNet-3D stem after space-to-depth (CS = 8)
    (3, 10, 11, 12, 8, 16, (3, 3, 3), "same"),       # CS = 8, 27 taps (last k-step partial), padding
]


@pytest.mark.parametrize("case", CASES)
def test_conv_tile_fwd_dgrad(case, monkeypatch):
    assert _native.kernels_available(), "HIP kernel library (_C) must be built and loadable on the GPU box"
    N, D, H, W, C, K, k, pad = case
    torch.manual_seed(0)
    dev = "cuda"
    x = torch.randn(N, D, H, W, C, device=dev).to(torch.bfloat16)
    spec = ConvSpec.make(x.shape, K, k, 1, pad)
    w = (torch.randn(K, spec.KD, spec.KH, spec.KW, C, device=dev) * 0.05).to(torch.bfloat16).float()
    b = torch.randn(K, device=dev) * 0.1
    pf, pd = ct.fwd_plan(spec), ct.dgrad_plan(spec)
    assert pf is not None and (pd is not None or C < 16), (pf, pd)   # dgrad needs >= 16 output columns

    # forward with bias + relu
    y, _ = ct.conv_fwd(x, w, b, spec, 1, False, pf)
    yr = torch.relu(ref.conv(x.float(), w, b, spec))
    l2, mx = _rel(y, yr)
    assert l2 < 8e-3 and mx < 2e-2, (l2, mx)

    # forward with BN statistics (no bias / act)
    y2, st = ct.conv_fwd(x, w, None, spec, 0, True, pf)
    y2r = ref.conv(x.float(), w, None, spec)
    l2, mx = _rel(y2, y2r)
    assert l2 < 8e-3 and mx < 2e-2, (l2, mx)
    s = st.sum(0)
    yb = y2.float().reshape(-1, K)
    torch.testing.assert_close(s[0], yb.sum(0), rtol=1e-3, atol=1e-2 * yb.abs().sum(0).max().item() / yb.shape[0])
    torch.testing.assert_close(s[1], (yb * yb).sum(0), rtol=1e-3, atol=1e-3)

    # dgrad: dx = conv_transpose(dy, w)
    if pd is None:
        return
    dy = torch.randn(spec.out_shape5, device=dev).to(torch.bfloat16)
    dx = ct.conv_dgrad(dy, w, spec, pd)
    xr = x.float().clone().requires_grad_(True)
    yr = ref.conv(xr, w, None, spec)
    (gx,) = torch.autograd.grad(yr, xr, dy.float())
    l2, mx = _rel(dx, gx)
    assert l2 < 8e-3 and mx < 2e-2, (l2, mx)


def test_conv_tile_repeatable_and_counters_reset():
    """Back-to-back launches on one stream reuse the schedule counters (each launch leaves
    them zero) and give bit-identical outputs."""
    torch.manual_seed(1)
    x = torch.randn(8, 25, 25, 25, 32, device="cuda").to(torch.bfloat16)
    spec = ConvSpec.make(x.shape, 64, (4, 4, 4), 1, "valid")
    w = (torch.randn(64, 4, 4, 4, 32, device="cuda") * 0.05).float()
    p = ct.fwd_plan(spec)
    outs = [ct.conv_fwd(x, w, None, spec, 0, False, p)[0] for _ in range(3)]
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])
    assert int(ct.sched(x.device, _native.stream(x)).abs().sum()) == 0
