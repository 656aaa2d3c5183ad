"""CPU emulation of the implicit-GEMM gather (tap tables + weight packing).

The HIP kernels read ``A[m][k]`` through per-layer tap tables built in
``featurenet_amd/ops/conv.py``.  This test re-implements the kernel's
``gather8`` in numpy for all three gather modes (scalar / 16-B vector /
packed-W) and the transposed (dgrad) table, multiplies by the packed weight
operand and compares with the PyTorch reference convolution -- so table or
packing bugs are caught on CPU, before a kernel ever reads out of bounds.
"""
import numpy as np
import pytest
import torch

import importlib

C = importlib.import_module("featurenet_amd.ops.conv")
from featurenet_amd.ops import reference as ref
from featurenet_amd.ops.spec import ConvSpec


def _rows(geom, M):
    RD, RH, RW, md, mh, mw, ad, ah, aw, SD, SH, SW, SC, kwc = geom
    m = np.arange(M)
    c3 = m % RW
    t = m // RW
    c2 = t % RH
    t //= RH
    c1 = t % RD
    n = t // RD
    bd, bh, bw = c1 * md + ad, c2 * mh + ah, c3 * mw + aw
    base = (((n * SD + bd) * SH + bh) * SW + bw) * SC
    return base, bd, bh, bw


def emulate_A(src_flat, tab, geom, M, Kdim, gm):
    RD, RH, RW, md, mh, mw, ad, ah, aw, SD, SH, SW, SC, kwc = geom
    base, bd, bh, bw = _rows(geom, M)
    A = np.zeros((M, Kdim), dtype=np.float64)
    nchunks = (Kdim + 7) // 8
    for kc in range(nchunks):
        for j in range(8):
            k = kc * 8 + j
            if k >= Kdim:
                continue
            if gm == C.GM_SCALAR:
                off, zd, zh, zw = tab[k]
                ok = (bd + zd >= 0) & (bd + zd < SD) & (bh + zh >= 0) & (bh + zh < SH) & (bw + zw >= 0) & (bw + zw < SW)
                idx = base + off
            elif gm == C.GM_VEC:
                off, zd, zh, zw = tab[kc]
                ok = (bd + zd >= 0) & (bd + zd < SD) & (bh + zh >= 0) & (bh + zh < SH) & (bw + zw >= 0) & (bw + zw < SW)
                idx = base + off + j
            else:
                off, dh, lh, p0 = tab[kc]
                zd, zh = dh >> 16, dh & 0xFFFF
                lo, hi = lh >> 16, lh & 0xFFFF
                rowok = (bd + zd >= 0) & (bd + zd < SD) & (bh + zh >= 0) & (bh + zh < SH)
                fast = rowok & (bw + lo >= 0) & (bw + hi < SW)
                pp = p0 + j
                kw = pp // SC
                slow = rowok & ~fast & (pp < kwc) & (bw + kw >= 0) & (bw + kw < SW)
                ok = fast | slow
                idx = base + off + j
                # the fast path must stay inside the tensor for every lane
                assert np.all(idx[fast] < src_flat.size) and np.all(idx[fast] >= 0)
            vals = np.zeros(M)
            vals[ok] = src_flat[idx[ok]]
            A[:, k] = vals
    return A


CASES = [
    (2, 9, 9, 9, 8, 16, (3, 3, 3), 1, "valid"),
    (2, 12, 12, 12, 1, 8, (5, 5, 5), 2, "valid"),     # conv1-like, packed-W
    (2, 1, 11, 13, 3, 6, (1, 5, 5), 1, "same"),        # RGB first layer, packed-W + padding fallback
    (2, 1, 10, 10, 3, 6, (1, 3, 3), 2, "same"),
    (1, 1, 7, 9, 5, 4, (1, 3, 1), 1, "same"),          # scalar mode (C=5 with KW=1 -> packed)
    (2, 1, 8, 8, 12, 4, (1, 3, 3), 1, "same"),         # scalar mode (C=12)
]


@pytest.mark.parametrize("case", CASES)
def test_forward_gather_matches_reference(case):
    N, D, H, W, Cin, K, k, s, pad = case
    torch.manual_seed(0)
    x = torch.randn(N, D, H, W, Cin, dtype=torch.float64)
    spec = ConvSpec.make(x.shape, K, k, s, pad)
    # bf16-representable weights: the packed operand is bf16
    w = torch.randn(K, spec.KD, spec.KH, spec.KW, Cin).bfloat16().double()
    gm = C.gather_mode(spec)
    tab = (C._packw_table(spec) if gm == C.GM_PACKW else C._fwd_table(spec, gm == C.GM_VEC)).astype(np.int64)
    kd = C.kdim_gather(spec)
    A = emulate_A(x.numpy().ravel(), tab, C._geom_fwd(spec), spec.M, kd, gm)
    wm, ld = C.pack_weight_rows(w.float(), spec)
    Bm = wm.double().numpy()[:, :kd]
    if gm != C.GM_PACKW:
        Bm = w.reshape(K, -1).numpy()
    y = (A @ Bm.T).reshape(spec.out_shape5)
    yr = ref.conv(x, w, None, spec).numpy()
    np.testing.assert_allclose(y, yr, rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("case", [c for c in CASES if c[4] % 8 == 0 or True])
def test_dgrad_gather_matches_autograd(case):
    N, D, H, W, Cin, K, k, s, pad = case
    torch.manual_seed(1)
    x = torch.randn(N, D, H, W, Cin, dtype=torch.float64, requires_grad=True)
    spec = ConvSpec.make(tuple(x.shape), K, k, s, pad)
    w = torch.randn(K, spec.KD, spec.KH, spec.KW, Cin, dtype=torch.float64)
    y = ref.conv(x, w, None, spec)
    g = torch.randn_like(y)
    y.backward(g)
    dy = g.detach().numpy()
    if spec.sd > 1 or spec.sh > 1 or spec.sw > 1:
        ODu, OHu, OWu = C._dgrad_src_dims(spec)
        up = np.zeros((N, ODu, OHu, OWu, K))
        up[:, :: spec.sd, :: spec.sh, :: spec.sw] = dy
        dy = up
    vec = spec.K % 8 == 0
    tab = C._dgrad_table(spec, vec).astype(np.int64)
    M = N * D * H * W
    A = emulate_A(dy.ravel(), tab, C._geom_dgrad(spec), M, spec.taps * K, C.GM_VEC if vec else C.GM_SCALAR)
    wt = w.reshape(K, spec.taps, Cin).permute(2, 1, 0).reshape(Cin, spec.taps * K).numpy()
    dx = (A @ wt.T).reshape(N, D, H, W, Cin)
    np.testing.assert_allclose(dx, x.grad.numpy(), rtol=1e-6, atol=1e-6)
