"""linear_infer (bf16 weight copy, inference FC layers) against an fp32 torch matmul: partial
row and column blocks, 64- and 128-column workgroups, single and split K (up to the 128^3 FC1's
1024-row batch; a 256-row workgroup variant measured slower there -- 2.53 vs 1.84 ms -- with
half the waves in flight, and was not kept)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K", [(1024, 128, 8192), (700, 100, 4096), (512, 64, 256), (300, 128, 2048),
                                   (1024, 128, 100000)])
@pytest.mark.parametrize("act", [None, "relu"])
def test_linear_infer_matches_fp32(M, N, K, act):
    from featurenet_amd.ops.linear import linear_infer

    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    y = linear_infer(x, w.contiguous(), b, act=act, out_fp32=True)
    ref = x.float() @ w.float().t() + b
    if act == "relu":
        ref = ref.clamp_min(0)
    err = ((y - ref).norm() / ref.norm()).item()
    assert err < 1e-3, err
