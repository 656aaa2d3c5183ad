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


@pytest.mark.parametrize("K", [6, 18, 1001, 64])
def test_dense_dgrad_any_k_is_native(K, monkeypatch):
    """Dense backward with an input width K that is not a multiple of 4 (a Dense fed by a Dense of
    width 6 or 18 in the NAS search space) runs the native dgrad kernel -- torch.matmul is never
    called -- and matches the fp32 reference."""
    from featurenet_amd.ops.linear import linear

    calls = {"matmul": 0}
    real = torch.matmul

    def spy(*a, **k):
        calls["matmul"] += 1
        return real(*a, **k)

    torch.manual_seed(K)
    dev = "cuda"
    x = torch.randn(37, K, device=dev).to(torch.bfloat16).requires_grad_(True)
    w = torch.nn.Parameter(torch.randn(24, K, device=dev) * 0.1)
    b = torch.nn.Parameter(torch.randn(24, device=dev) * 0.1)
    monkeypatch.setattr(torch, "matmul", spy)
    y = linear(x, w, b, "relu", out_fp32=True)
    g = torch.randn_like(y)
    y.backward(g)
    monkeypatch.setattr(torch, "matmul", real)
    assert calls["matmul"] == 0
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    yr = torch.relu(xr @ wr.t() + b.detach())
    yr.backward(g)
    rel = ((x.grad.float() - xr.grad).norm() / xr.grad.norm()).item()
    assert rel < 1e-2, rel
    relw = ((w.grad - wr.grad).norm() / wr.grad.norm()).item()
    assert relw < 1e-2, relw


def test_dense_softmax_activation_native():
    """A Dense with a softmax activation: the native row-softmax forward and backward against
    torch's fp32 softmax."""
    from featurenet_amd.ops.linear import linear

    torch.manual_seed(3)
    dev = "cuda"
    for N in (10, 100, 300):
        x = torch.randn(53, 40, device=dev).to(torch.bfloat16)
        w = torch.nn.Parameter(torch.randn(N, 40, device=dev) * 0.2)
        y = linear(x, w, None, "softmax")
        g = torch.randn_like(y)
        y.backward(g)
        wr = w.detach().clone().requires_grad_(True)
        yr = torch.softmax(x.float() @ wr.t(), dim=-1)
        yr.backward(g)
        assert torch.allclose(y.sum(-1), torch.ones(53, device=dev), atol=1e-5)
        assert (y - yr).abs().max().item() < 2e-2
        rel = ((w.grad - wr.grad).norm() / wr.grad.norm()).item()
        assert rel < 2e-2, (N, rel)
