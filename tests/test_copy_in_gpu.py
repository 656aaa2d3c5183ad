"""_native.copy_in: the step's batch copy-in as one launch -- exact for both buffers, odd byte
counts (tail bytes), and the torch fallback for unaligned views."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n0,n1", [(128 * 64 ** 3, 128), (1000003, 17), (16, 0), (4096, 4096 * 3 + 5)])
def test_copy_in_exact(n0, n1):
    from featurenet_amd import _native

    g = torch.Generator(device="cuda").manual_seed(0)
    s0 = torch.randint(0, 256, (n0,), dtype=torch.uint8, device="cuda", generator=g)
    d0 = torch.zeros_like(s0)
    if n1:
        s1 = torch.randint(0, 1 << 30, (n1,), dtype=torch.int64, device="cuda", generator=g)
        d1 = torch.zeros_like(s1)
        _native.copy_in(d0, s0, d1, s1)
    else:
        _native.copy_in(d0, s0)
    torch.cuda.synchronize()
    assert torch.equal(d0, s0)
    if n1:
        assert torch.equal(d1, s1)


def test_copy_in_unaligned_falls_back():
    from featurenet_amd import _native

    s = torch.arange(1000, dtype=torch.uint8, device="cuda")
    d = torch.zeros(1001, dtype=torch.uint8, device="cuda")
    _native.copy_in(d[1:], s)                       # (1-byte offset: torch's copy)
    torch.cuda.synchronize()
    assert torch.equal(d[1:], s)
