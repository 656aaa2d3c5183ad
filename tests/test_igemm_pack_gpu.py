"""One-launch B-operand packing of the gather conv kernels (``igemm_pack_w``) against the
torch formulation it replaced (cast, transpose, zero rows / channels, padded row stride),
and a channel-padded conv (C, Cout % 8 != 0) through the whole native path against fp32."""
import dataclasses

import pytest
import torch

pytestmark = pytest.mark.gpu

from featurenet_amd import _native  # noqa: E402
from featurenet_amd.ops import reference as ref  # noqa: E402
from featurenet_amd.ops.spec import ConvSpec  # noqa: E402

import importlib  # noqa: E402

CV = importlib.import_module("featurenet_amd.ops.conv")


def _torch_pack(w, spec, mode):
    w = CV.pad_to_spec(w.float(), spec)
    if mode == 1:
        mat = w.reshape(spec.K, spec.taps, spec.C).permute(2, 1, 0).reshape(spec.C, spec.taps * spec.K)
    elif mode == 2:
        R = CV.packw_row(spec)
        out = torch.zeros(spec.K, spec.KD * spec.KH, R, device=w.device)
        out[:, :, :spec.KW * spec.C] = w.reshape(spec.K, spec.KD * spec.KH, spec.KW * spec.C)
        return out.reshape(spec.K, -1).to(torch.bfloat16)
    else:
        mat = w.reshape(spec.K, spec.kdim)
    ld = (mat.shape[1] + 7) // 8 * 8
    out = torch.zeros(mat.shape[0], ld, device=w.device)
    out[:, :mat.shape[1]] = mat
    return out.to(torch.bfloat16)


@pytest.mark.parametrize("K0,C0,K,Cp,k,mode", [(6, 3, 6, 3, 5, 0), (16, 6, 16, 8, 5, 0), (10, 12, 16, 16, 3, 1),
                                               (6, 3, 6, 3, 5, 2), (120, 16, 120, 16, 5, 1)])
def test_igemm_pack_w_modes(K0, C0, K, Cp, k, mode):
    assert _native.kernels_available()
    torch.manual_seed(0)
    w = torch.randn(K0, 1, k, k, C0, device="cuda")
    spec = ConvSpec.make((2, 1, 12, 12, Cp), K, (1, k, k), 1, "same")
    got, ld = CV._native_pack(w, spec, mode)
    exp = _torch_pack(w, spec, mode)
    assert got.shape == exp.shape, (got.shape, exp.shape)
    assert torch.equal(got, exp)


def test_channel_padded_conv_grads_match_fp32():
    """C = 6, Cout = 10 (both padded to 8 / 16 internally): forward, dx, dW, db vs fp32 torch."""
    torch.manual_seed(1)
    x = torch.randn(4, 1, 20, 20, 6, device="cuda").to(torch.bfloat16)
    spec = ConvSpec.make(tuple(x.shape), 10, (1, 5, 5), 1, "same")
    w = (torch.randn(10, 1, 5, 5, 6, device="cuda") * 0.1).requires_grad_(True)
    b = (torch.randn(10, device="cuda") * 0.1).requires_grad_(True)
    xg = x.clone().requires_grad_(True)
    y = CV.conv(xg, w, b, spec, "relu")
    dy = torch.randn_like(y.float())
    y.float().backward(dy)
    xr = x.float().clone().requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    yr = ref.conv(xr, wr, br, spec, "relu")
    yr.backward(dy)

    def rel(a, r):
        return ((a.float() - r).norm() / (r.norm() + 1e-12)).item()
    assert rel(y, yr) < 1e-2
    assert rel(xg.grad, xr.grad) < 2e-2
    assert rel(w.grad, wr.grad) < 2e-2
    assert rel(b.grad, br.grad) < 2e-2
