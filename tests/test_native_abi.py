"""Python <-> _C argument plumbing, checked on CPU.

The HIP entry points cannot run here, but their pybind11 signatures can:
every op-layer call is routed to a fake module whose functions enforce the
arity of the real ``_C`` function (parsed from its pybind docstring), so a
mismatch between ops/*.py and bind.cpp fails in the CPU suite instead of on
the GPU box.
"""
import re

import pytest
import torch

from featurenet_amd import _native


def _arity(fn) -> tuple[int, int]:
    """(required, total) parameter counts from the pybind11 signature line."""
    sig = fn.__doc__.split("\n")[0]
    inner = sig[sig.index("(") + 1:sig.rindex(") ->")] if ") ->" in sig else sig[sig.index("(") + 1:sig.rindex(")")]
    depth, parts, cur = 0, [], ""
    for ch in inner:
        depth += ch in "[(" and 1 or 0
        depth -= ch in "])" and 1 or 0
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        parts.append(cur)
    return sum("=" not in p for p in parts), len(parts)


class _FakeK:
    def __init__(self, real):
        self.real, self.calls = real, []

    def __getattr__(self, name):
        real_fn = getattr(self.real, name)
        lo, hi = _arity(real_fn)

        def f(*args):
            assert lo <= len(args) <= hi, f"{name}: called with {len(args)} args, binding takes {lo}..{hi}"
            self.calls.append(name)
            if name.endswith(("_lds", "mblocks", "_workers", "_blocks", "_yblocks", "_gx", "_part", "_splits")):
                return 1
            return None
        return f


@pytest.fixture()
def fake(monkeypatch):
    if not _native.kernels_available():
        pytest.skip("_C not built")
    fk = _FakeK(_native.kernels())
    monkeypatch.setattr(_native, "kernels", lambda: fk)
    monkeypatch.setattr(_native, "stream", lambda t=None: 0)
    return fk


def test_halo_calls_match_bindings(fake):
    import importlib

    C = importlib.import_module("featurenet_amd.ops.conv")
    x = torch.zeros(2, 29, 29, 29, 32, dtype=torch.bfloat16)
    spec = C.ConvSpec.make(x.shape, 32, 5)
    w = torch.zeros(32, 5, 5, 5, 32)
    C.halo_conv_fwd(x, w, None, spec, 0, True, C.halo_fwd_plan(spec))
    C.halo_conv_fwd(x, w, torch.zeros(32), spec, 1, False, C.halo_fwd_plan(spec))
    dy = torch.zeros(spec.out_shape5, dtype=torch.bfloat16)
    C.halo_conv_dgrad(dy, w, spec, C.halo_dgrad_plan(spec))
    C.halo_conv_wgrad(dy, x, spec, C.halo_wgrad_plan(spec))
    assert fake.calls.count("conv_halo") == 3 and "conv_halo_wgrad" in fake.calls


def test_igemm_and_misc_calls_match_bindings(fake):
    import importlib

    C = importlib.import_module("featurenet_amd.ops.conv")
    x = torch.zeros(2, 16, 16, 16, 1, dtype=torch.bfloat16)
    spec = C.ConvSpec.make(x.shape, 32, 7, 2)
    wm, ld = C.pack_weight_rows(torch.zeros(32, 7, 7, 7, 1), spec)
    C.native_conv_fwd(x, wm, ld, None, spec, 0, True)
    dy = torch.zeros(spec.out_shape5, dtype=torch.bfloat16)
    C.native_conv_wgrad(dy, x, spec)
    C.native_colsum(torch.zeros(64, 32, dtype=torch.bfloat16))
    xs = torch.zeros(2, 1, 9, 9, 8, dtype=torch.bfloat16)
    ds = C.ConvSpec.make(xs.shape, 8, (1, 3, 3), 1, "same")
    y = C.DepthwiseFn.forward(type("Ctx", (), {"save_for_backward": lambda self, *a: None})(), xs,
                              torch.zeros(8, 1, 3, 3, 1), None, ds, 0)
    assert y.shape == (2, 1, 9, 9, 8)
    from featurenet_amd.ops.loss import SoftmaxXentFn

    SoftmaxXentFn.forward(type("Ctx", (), {"save_for_backward": lambda self, *a: None,
                                           "mark_non_differentiable": lambda self, *a: None})(),
                          torch.zeros(6, 25, dtype=torch.bfloat16), torch.zeros(6, dtype=torch.long), 0.0, True)
    assert {"igemm_fwd", "igemm_wgrad", "colstats", "bn_finalize", "dw_fwd", "softmax_xent_rows"} <= set(fake.calls)


def test_fp8_inference_calls_match_bindings(fake, monkeypatch):
    from featurenet_amd.inference.fp8 import Fp8Conv, quantize_fp8_act
    from featurenet_amd.models.layers import Conv

    conv = Conv(32, 64, (3, 3, 3), 1, "valid", bias=True)
    layer = Fp8Conv(conv, 0.02, 0.05)
    xq = torch.zeros(2, 10, 10, 10, 32, dtype=torch.uint8)
    y, shape = layer(xq, tuple(xq.shape))                      # fp8 tile kernel
    assert shape == (2, 8, 8, 8, 64) and y.dtype == torch.uint8
    monkeypatch.setenv("FN_F8_TILE", "0")
    y, shape = layer(xq, tuple(xq.shape))                      # fp8 halo kernel
    assert shape == (2, 8, 8, 8, 64) and y.dtype == torch.uint8
    quantize_fp8_act(torch.zeros(4, 8, dtype=torch.bfloat16), 0.1)
    assert {"conv_tile_f8", "conv_halo_f8", "quant_fp8"} <= set(fake.calls)


def test_fp8_block_scaled_calls_match_bindings(fake):
    from featurenet_amd.inference.fp8 import Fp8Conv, quantize_fp8_block
    from featurenet_amd.models.layers import Conv
    from featurenet_amd.ops import conv_tile

    conv = Conv(32, 64, (3, 3, 3), 1, "valid", bias=True)
    layer = Fp8Conv(conv, 1.0, 1.0)
    xq, xs = quantize_fp8_block(torch.zeros(2, 10, 10, 10, 32, dtype=torch.bfloat16))
    assert xq.dtype == torch.uint8 and xs.shape == (2, 10, 10, 10)
    (yq, ys), shape = layer((xq, xs), tuple(xq.shape))         # block-scaled in and out
    assert shape == (2, 8, 8, 8, 64) and ys.shape == (2, 8, 8, 8)
    from featurenet_amd.ops.spec import ConvSpec

    spec = ConvSpec.make((2, 12, 12, 12, 8), 32, 4, 1, "valid")      # (a space-to-depth stem shape)
    tp = conv_tile.fwd_plan(spec)
    yq, ys = conv_tile.conv_fwd_q8_block(torch.zeros(2, 12, 12, 12, 8, dtype=torch.bfloat16),
                                         torch.zeros(32, 4, 4, 4, 8), torch.zeros(32), spec, 1, tp)
    assert ys.shape == (2, 9, 9, 9)
    assert {"conv_tile_f8", "quant_fp8_block", "conv_tile"} <= set(fake.calls)


def test_halo_extent_check_rejects_undersized_tensors():
    """bind.cpp validates operand extents implied by the geometry before any HIP call."""
    if not _native.kernels_available():
        pytest.skip("_C not built")
    K = _native.kernels()
    geom = [2, 29, 29, 29, 32, 25, 25, 25, 5, 5, 5, 0, 0, 0, 1, 10, 25]
    src = 2 * 29 ** 3 * 32
    out = 2 * 25 ** 3 * 32
    wt = 32 * 32 * 128   # 125 taps padded to 128 (8 taps per 128-k stage)
    with pytest.raises(RuntimeError, match="src has"):
        K.conv_halo(0, 0, 0, 0, 0, 0, geom, 32, 0, 0, 0, [src - 1, wt, out, 128])
    with pytest.raises(RuntimeError, match="wt has"):
        K.conv_halo(0, 0, 0, 0, 0, 0, geom, 32, 0, 0, 0, [src, wt - 8, out, 128])
    with pytest.raises(RuntimeError, match="out has"):
        K.conv_halo(0, 0, 0, 0, 0, 0, geom, 32, 0, 0, 0, [src, wt, out // 2, 128])
    with pytest.raises(RuntimeError, match="dw has"):
        K.conv_halo_wgrad(0, 0, 0, 0, geom, 32, 1, 0, [out, src, 32 * 125 * 32 - 1, 32 * 125 * 32])
    bad = list(geom)
    bad[5] = 40                                           # output larger than the input allows
    with pytest.raises(RuntimeError, match="larger than"):
        K.conv_halo(0, 0, 0, 0, 0, 0, bad, 32, 0, 0, 0, [src, wt, out, 128])
    pg = [2, 20, 20, 20, 64, 10, 10, 10, 2, 2, 2, 2, 2, 2, 0, 0, 0]
    with pytest.raises(RuntimeError, match="out has"):
        K.pool_fwd(0, 0, 0, 0, pg, 1, 0, 0, 0, [2 * 8000 * 64, 100])
