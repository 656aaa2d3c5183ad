"""Binary voxel input as uint8 (the bench's data format): the space-to-depth stem packing reads the
bytes directly (``s2d_pack_kernel<unsigned char>``), and a training step gives the same bits as
with the same voxels in bf16 -- FeatureNet-3D (unpadded stride-2 stem, the packing's fast path)
and the segmentation model (padded stem, the general path)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _step(m, x, y, seg):
    from featurenet_amd.ops import softmax_xent

    m.zero_grad(set_to_none=True)
    loss = m.loss(x, y) if seg else softmax_xent(m(x), y)
    loss.backward()
    torch.cuda.synchronize()
    return loss.detach().clone(), {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("seg", [False, True])
def test_uint8_voxels_match_bf16(seg):
    from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DSeg

    torch.manual_seed(0)
    m = (FeatureNet3DSeg(input_size=32, num_classes=5) if seg else FeatureNet3D()).cuda().train()
    S = 32 if seg else 64
    occ = torch.rand(4, S, S, S, 1, device="cuda") < 0.3
    y = torch.randint(0, 5 if seg else 24, (4, S, S, S) if seg else (4,), device="cuda")
    a = _step(m, occ.to(torch.bfloat16), y, seg)
    b = _step(m, occ.to(torch.uint8), y, seg)
    assert torch.equal(a[0], b[0]), (a[0].item(), b[0].item())
    for n in a[1]:
        assert torch.equal(a[1][n], b[1][n]), n


def test_s2d_pack_uint8_matches_bf16():
    from featurenet_amd.ops.conv import s2d_input, s2d_plan
    from featurenet_amd.ops.spec import ConvSpec

    for shape, pad in (((2, 64, 64, 64, 1), "valid"), ((2, 32, 32, 32, 1), "same")):
        spec = ConvSpec.make(shape, 32, (7, 7, 7), (2, 2, 2), pad)
        f, spec2 = s2d_plan(spec)
        occ = torch.rand(*shape, device="cuda") < 0.4
        pads = (spec.pd, spec.ph, spec.pw)
        assert torch.equal(s2d_input(occ.to(torch.uint8), f, spec2, pads), s2d_input(occ.to(torch.bfloat16), f, spec2, pads))
