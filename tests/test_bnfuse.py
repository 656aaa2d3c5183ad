"""CPU checks of the BN-backward fusion hand-off (ops/bnfuse.py): matches only the exact
(z, y) pair, misses fall back, dead tensors never match."""
import gc

import torch

from featurenet_amd.ops import bnfuse


def test_source_and_take_match_only_the_tagged_pair(monkeypatch):
    y = torch.randn(2, 4, 4, 4, 8)
    prm = torch.randn(4, 8)
    z = torch.relu(y)
    mask = torch.zeros(z.numel() // 8, dtype=torch.uint8)
    bnfuse.tag_output(z, y, prm, 1, mask)
    src = bnfuse.source_of(z.reshape(2, 4, 4, 4, 8))      # a same-extent view matches
    assert src is not None and src[0] is y and src[1] is prm and src[2] == 1 and src[3] is mask
    assert bnfuse.source_of(torch.empty_like(z)) is None  # another tensor does not
    dz = torch.randn_like(z)
    slab = ("identity", torch.randn(3, 2, 8), torch.randn(2, 8))
    bnfuse.offer(dz, slab, y)
    assert bnfuse.take(dz, torch.empty_like(y)) is None   # wrong y: no slab (and the entry is consumed)
    bnfuse.offer(dz, slab, y)
    assert bnfuse.take(dz, y) is slab
    assert bnfuse.take(dz, y) is None                     # taken once


def test_dead_outputs_do_not_match(monkeypatch):
    y = torch.randn(64)
    prm = torch.randn(4, 1)
    z = torch.relu(y)
    ptr = z.data_ptr()
    bnfuse.tag_output(z, y, prm, 1, torch.zeros(8, dtype=torch.uint8))
    del z
    gc.collect()
    w = torch.empty(64)
    if w.data_ptr() == ptr:                               # allocator reuse must not resurrect the entry
        assert bnfuse.source_of(w) is None
    z2 = torch.relu(y)
    bnfuse.tag_output(z2, y, prm, 1)
    assert bnfuse.source_of(z2) is None                   # no relu mask (no identity path): nothing recorded


def test_identity_tag_keeps_mask(monkeypatch):
    monkeypatch.setenv("FN_BN_IDENTITY", "1")
    y = torch.randn(2, 4, 4, 4, 32)
    prm = torch.randn(4, 32)
    z = torch.relu(y)
    mask = torch.zeros(z.numel() // 8, dtype=torch.uint8)
    bnfuse.tag_output(z, y, prm, 1, mask)
    src = bnfuse.source_of(z)
    assert src is not None and src[3] is mask               # the identity path tags with the mask
    assert bnfuse.identity_ok(32, 1) and bnfuse.identity_ok(64, 1)
    assert not bnfuse.identity_ok(16, 1) and not bnfuse.identity_ok(32, 0)   # whole mask dwords; relu only
    monkeypatch.setenv("FN_BN_IDENTITY", "0")
    assert not bnfuse.identity_ok(32, 1)


def test_statistics_identity_math():
    """The algebra behind bn_bwd_prep_kernel, in float64 on the CPU: for z = relu(bn(y)) feeding
    a conv, sum_p dz*z = sum W*dW per input channel, and the apply constants built from it (no
    division by gamma) give autograd's BN input gradient -- including gamma <= 0."""
    import torch.nn.functional as F

    torch.manual_seed(0)
    N, C, K, S = 2, 4, 3, 7
    y = torch.randn(N, C, S, S, S, dtype=torch.float64) * 2 + 0.5
    gamma = torch.tensor([1.3, -0.7, 1e-6, 0.0], dtype=torch.float64)
    beta = torch.tensor([0.2, 0.9, -0.4, 0.6], dtype=torch.float64)
    W = torch.randn(K, C, 3, 3, 3, dtype=torch.float64)
    y.requires_grad_(True)
    z = F.batch_norm(y, None, None, gamma, beta, training=True, eps=1e-5).relu()
    zl = z.detach().requires_grad_(True)
    Wl = W.clone().requires_grad_(True)
    out = F.conv3d(zl, Wl)
    gout = torch.randn_like(out)
    dz, dW = torch.autograd.grad(out, (zl, Wl), gout)
    S_lhs = (dz * zl.detach()).sum(dim=(0, 2, 3, 4))
    S_rhs = (W * dW).sum(dim=(0, 2, 3, 4))
    assert torch.allclose(S_lhs, S_rhs, rtol=1e-10, atol=1e-9)
    (dy_ref,) = torch.autograd.grad(z, y, dz)
    # the kernel's formula
    M = N * S ** 3
    mean = y.detach().mean(dim=(0, 2, 3, 4))
    var = y.detach().var(dim=(0, 2, 3, 4), unbiased=False)
    invstd = 1.0 / torch.sqrt(var + 1e-5)
    scale = gamma * invstd
    g = dz * (z.detach() > 0)
    sg = g.sum(dim=(0, 2, 3, 4))
    G = S_rhs - beta * sg
    k1 = scale
    k2 = -invstd ** 2 * G / M
    k3 = -scale * sg / M + mean * invstd ** 2 * G / M
    sh = (1, C, 1, 1, 1)
    dy = k1.view(sh) * g + k2.view(sh) * y.detach() + k3.view(sh)
    assert torch.allclose(dy, dy_ref, rtol=1e-8, atol=1e-10)
