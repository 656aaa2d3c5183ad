"""Column sums for channel counts that are not a multiple of 8 (super-row vector path of
colstats) and the loss backward's device-side dloss scale, against fp32 PyTorch."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from featurenet_amd import _native  # noqa: E402


@pytest.mark.parametrize("M,C", [(4096, 25), (8192, 12), (1000, 3), (2048, 24), (64 * 1024, 25), (4096, 250)])
def test_colsum_matches_torch(M, C):
    from featurenet_amd.ops.conv import native_colsum

    assert _native.kernels() is not None
    torch.manual_seed(0)
    x = torch.randn(M, C, device="cuda").to(torch.bfloat16)
    got = native_colsum(x)
    ref = x.float().sum(0)
    assert torch.allclose(got, ref, rtol=1e-4, atol=1e-2 * (M ** 0.5) * 1e-2), (got - ref).abs().max()


@pytest.mark.parametrize("scale", [1.0, 2.5])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_softmax_xent_backward_scales_by_dloss(scale, dtype):
    from featurenet_amd.ops import softmax_xent

    torch.manual_seed(1)
    logits = torch.randn(512, 25, device="cuda").to(dtype).requires_grad_(True)
    labels = torch.randint(0, 25, (512,), device="cuda")
    (softmax_xent(logits, labels) * scale).backward()
    ref_logits = logits.detach().float().requires_grad_(True)
    (torch.nn.functional.cross_entropy(ref_logits, labels) * scale).backward()
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    assert torch.allclose(logits.grad.float(), ref_logits.grad, rtol=tol, atol=tol * 1e-2 * scale)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_softmax_xent_second_backward_with_scaled_dloss(dtype):
    """retain_graph: a second backward after a first one whose upstream gradient was not 1
    must not see the first call's scale (the first backward scales d(logits) in place)."""
    from featurenet_amd.ops import softmax_xent

    torch.manual_seed(2)
    logits = torch.randn(300, 24, device="cuda").to(dtype).requires_grad_(True)
    labels = torch.randint(0, 24, (300,), device="cuda")
    loss = softmax_xent(logits, labels)
    g1, = torch.autograd.grad(loss * 2.0, logits, retain_graph=True)
    g2, = torch.autograd.grad(loss * 3.0, logits)
    ref_logits = logits.detach().float().requires_grad_(True)
    base, = torch.autograd.grad(torch.nn.functional.cross_entropy(ref_logits, labels), ref_logits)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    assert torch.allclose(g1.float(), 2.0 * base, rtol=tol, atol=tol * 2e-2)
    assert torch.allclose(g2.float(), 3.0 * base, rtol=tol, atol=tol * 3e-2)
