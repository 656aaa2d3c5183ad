"""FP8 inference for FeatureNet-3D (BASELINE config 5: 128^3 voxels, batch 1024).

Post-training quantisation, inference only:

* BatchNorm is folded into the conv weights and bias (eval statistics);
* weights are quantised per output channel to OCP e4m3 (amax / 448);
* activations between layers are OCP MX-style block-scaled e4m3 (default, ``FN_F8_BLOCK=1``): every
  (position, 32-channel block) carries its own E8M0 power-of-two scale, written by the producing
  epilogue (``osc``) and applied inside ``v_mfma_scale_f32_16x16x128_f8f6f4`` by the consumer (its
  loader LDS-DMAs the scale dwords with each halo) -- no calibration, and a position with small
  activations keeps e4m3's full relative precision however large the tensor's maximum is;
  ``FN_F8_BLOCK=0`` (or a shape without a block-scaled tile plan) quantises per tensor with scales
  calibrated from a bf16 forward pass (``amax / 448`` of each layer's post-ReLU output);
* conv2..conv4 run the fp8 variant of the big-tile kernel (``conv_tile.hip``,
  ``conv_tile_kernel<8, 2, CPP, 0, true>``: LDS-DMA'd e4m3 halo, weights streamed in
  MFMA-fragment order, ``v_mfma_scale_f32_16x16x128_f8f6f4``, dequantise + bias + ReLU
  (+ requantise) from registers), or ``conv_halo_f8`` (``csrc/kernels/conv_fp8.hip``): fp8
  halo tiles in LDS, block-scaled ``mfma_scale_f32_16x16x128_f8f6f4``, dequantise + bias + ReLU
  (+ requantise to fp8) in the epilogue.  conv1 (1-channel, stride 2) stays on
  the bf16 path (space-to-depth tile kernel) with the folded BN + ReLU fused,
  followed by one quantisation pass; conv4 writes bf16 for the max-pool and the
  two dense layers (native split-K MFMA kernels on bf16 weight copies, 128-column
  workgroups: ``csrc/kernels/dense.hip``).
"""
from __future__ import annotations

import math
import os
import warnings

import torch

from .. import _native
from .. import ops
from ..models.featurenet3d import FeatureNet3D
from ..ops import conv_tile
from ..ops.conv import halo_plan, halo_tap_offsets
from ..ops.spec import ConvSpec, PoolSpec

FP8_MAX = 448.0
I8_MAX = 127.0
AGREEMENT_WARN = 0.97      # calibration-set top-1 agreement below which quantize_model warns
FALLBACK_AT = 0.99         # quantize_model(fallback=True): the agreement each fallback step must reach


def _fold_bn(conv) -> tuple[torch.Tensor, torch.Tensor]:
    w = conv.weight.detach().float()
    if conv.bn:
        g = conv.gamma.detach().float() / torch.sqrt(conv.running_var.float() + conv.bn_eps)
        b = conv.beta.detach().float() - conv.running_mean.float() * g
        return w * g.view(-1, 1, 1, 1, 1), b
    b = conv.bias.detach().float() if conv.bias is not None else torch.zeros(w.shape[0], device=w.device)
    return w, b


def _to_fp8(t: torch.Tensor) -> torch.Tensor:
    return t.clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn)


class Fp8Conv:
    """One stride-1 conv layer on the fp8 tile kernel (``conv_tile.hip``, F8 variant) or the
    fp8 halo kernel (``conv_fp8.hip``: fallback for shapes the tile planner rejects, and the
    A/B reference); folded BN, per-channel weight scales.  ``FN_F8_TILE=0`` forces the halo
    kernel."""

    def __init__(self, conv, in_scale: float, out_scale: float | None, relu: bool = True, wb=None,
                 padding: str | None = None, int8: bool = False):
        # conv: the bf16 layer (BN folded here), or None with wb = (folded weight, bias)
        # int8: int8 operands (per-channel weights amax / 127; the input quantised with in_scale
        # the same way) on the tile kernel's int8 MFMA instance -- the binary-voxel stem
        w, b = _fold_bn(conv) if wb is None else wb
        K, KD, KH, KW, Cin = w.shape
        T = KD * KH * KW
        self.int8 = bool(int8)
        if self.int8:
            sw = w.abs().reshape(K, -1).amax(1).clamp_min(1e-12) / I8_MAX
            wq = torch.round(w / sw.view(-1, 1, 1, 1, 1)).clamp(-I8_MAX, I8_MAX).to(torch.int8)
            self.wq = None                                   # (tile kernel only)
        else:
            sw = w.abs().reshape(K, -1).amax(1).clamp_min(1e-12) / FP8_MAX
            wq = _to_fp8(w / sw.view(-1, 1, 1, 1, 1))
            # fp8 weights in the halo kernel's k order ([K][C/16][T8][16] bytes)
            T8 = (T + 7) // 8 * 8
            lay = torch.zeros(K, Cin // 16, T8, 16, dtype=torch.float8_e4m3fn, device=w.device)
            lay[:, :, :T] = wq.reshape(K, T, Cin // 16, 16).permute(0, 2, 1, 3)
            self.wq = lay.reshape(K, -1).view(torch.uint8).contiguous()
        self.wq_ktc = wq.reshape(K, T, Cin).view(torch.uint8).contiguous()   # [K][T][C] for the tile packing
        self._tile = {}
        self.scale = (in_scale * sw).float().contiguous()
        self.wscale = sw.float().contiguous()          # (block-scaled inputs: the weights' dequantisation only)
        self.bias = b.float().contiguous()
        self.out_scale, self.relu = out_scale, relu
        self.K, self.kernel, self.conv = K, (KD, KH, KW), conv
        self.padding = padding if padding is not None else conv.padding
        self.w_dequant = wq.float() * sw.view(-1, 1, 1, 1, 1)     # for numerics tests

    def tile_plan(self, spec, pool: bool = False, block: bool = False):
        if os.environ.get("FN_F8_TILE", "1") == "0":
            return None
        if block and (self.int8 or spec.C % 32 or spec.C > 128 or spec.K > 128):
            return None
        return conv_tile.plan(spec.N, (spec.OD, spec.OH, spec.OW), (spec.KD, spec.KH, spec.KW), spec.C, spec.K,
                              f8=True, pool=pool, bs=block)

    def pool_plan(self, shape5: tuple, block: bool = False):
        """The tile plan with the fused 2^3 max-pool epilogue for this input, or None."""
        if os.environ.get("FN_F8_POOL", "1") == "0" or self.out_scale is not None or not self.relu:
            return None
        return self.tile_plan(ConvSpec.make(shape5, self.K, self.kernel, 1, self.padding), pool=True, block=block)

    def __call__(self, xq, shape5: tuple, pool: bool = False) -> tuple:
        """(y, y's shape); ``pool``: y = maxpool2^3(relu(conv)) from the fused epilogue (the
        caller checked :meth:`pool_plan`).  Block-scaled mode: ``xq`` is ``(e4m3 bytes, scale
        dwords)`` and so is y unless it is the bf16 output of the last layer (tile kernel only)."""
        spec = ConvSpec.make(shape5, self.K, self.kernel, 1, self.padding)
        block = isinstance(xq, tuple)
        tp = self.tile_plan(spec, pool=pool, block=block)
        if pool:
            assert tp is not None and tp.pool
        if block:
            if tp is None:
                raise RuntimeError(f"no block-scaled fp8 tile plan for {spec}")
            wpk = self._tile.get(tp)
            if wpk is None:
                wpk = self._tile[tp] = conv_tile.pack_weights_f8(self.wq_ktc, tp)
            out_block = self.out_scale is not None and not pool
            y = conv_tile.conv_fwd_f8(xq[0], wpk, self.wscale, self.bias, spec, tp, self.relu, None, xsc=xq[1],
                                      out_block=out_block)
            return y, tuple((y[0] if out_block else y).shape)
        if tp is not None:
            wpk = self._tile.get(tp)
            if wpk is None:
                wpk = self._tile[tp] = conv_tile.pack_weights_f8(self.wq_ktc, tp)
            y = conv_tile.conv_fwd_f8(xq, wpk, self.scale, self.bias, spec, tp, self.relu, self.out_scale,
                                      i8=self.int8)
            return y, tuple(y.shape)
        if self.int8:
            raise RuntimeError(f"no int8 tile plan for {spec}")
        # fp8 halo = 16 B/position; halo_plan counts 32 B/position (bf16): <= 64 KiB of fp8 halo
        plan = halo_plan(spec.OD, spec.OH, spec.OW, spec.KD, spec.KH, spec.KW, 128 * 1024, wsplit=False)
        if plan is None:
            raise RuntimeError(f"no fp8 halo tile for {spec}")
        geom = [spec.N, spec.D, spec.H, spec.W, spec.C, spec.OD, spec.OH, spec.OW, spec.KD, spec.KH, spec.KW,
                spec.pd, spec.ph, spec.pw, plan[0], plan[1]]
        out_f8 = self.out_scale is not None
        y = torch.empty(spec.out_shape5, dtype=torch.uint8 if out_f8 else torch.bfloat16, device=xq.device)
        toffs = halo_tap_offsets(geom, xq.device)
        _native.kernels().conv_halo_f8(xq.data_ptr(), self.wq.data_ptr(), self.scale.data_ptr(),
                                       self.bias.data_ptr(), y.data_ptr(),
                                       1.0 / self.out_scale if out_f8 else 1.0, toffs.data_ptr(), geom, self.K,
                                       int(out_f8), int(self.relu), _native.stream(xq))
        return y, spec.out_shape5


def quantize_fp8_act(x: torch.Tensor, scale: float) -> torch.Tensor:
    """bf16 activation -> fp8 bytes of x / scale (native kernel)."""
    y = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    _native.kernels().quant_fp8(x.data_ptr(), y.data_ptr(), x.numel(), 1.0 / scale, _native.stream(x))
    return y


def quantize_fp8_block(x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """bf16 channels-last activation [..., C] (C % 32 == 0, C <= 128) -> OCP MX-style block-scaled
    e4m3: (bytes [..., C], int32 scale dwords [...]: byte j = the E8M0 scale of channels 32j..)."""
    x = x.to(torch.bfloat16).contiguous()
    C = x.shape[-1]
    M = x.numel() // C
    y = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    sc = torch.zeros(x.shape[:-1], dtype=torch.int32, device=x.device)
    _native.kernels().quant_fp8_block(x.data_ptr(), y.data_ptr(), sc.data_ptr(), M, C, _native.stream(x),
                                      [x.numel(), y.numel(), sc.numel()])
    return y, sc


def dequantize_fp8_block(y: torch.Tensor, sc: torch.Tensor) -> torch.Tensor:
    """fp32 values of a block-scaled e4m3 tensor (:func:`quantize_fp8_block` layout)."""
    C = y.shape[-1]
    v = y.view(torch.float8_e4m3fn).float().reshape(*y.shape[:-1], C // 32, 32)
    e = ((sc.unsqueeze(-1) >> (8 * torch.arange(C // 32, device=sc.device))) & 255).float() - 127.0
    return (v * torch.exp2(e).unsqueeze(-1)).reshape(y.shape)


def stem_tap_plan(c1, in_shape5):
    """(ConvSpec of the tap-expanded stem, packed grid dims) when the stem -- 1 input channel,
    stride 2^3, 'valid', k^3 with ceil(k/2) = 4 -- can run as an fp8 conv: space-to-depth to
    8 channels, then the 4 w-taps of the packed grid folded into 32 channels
    (``s2d_tap_f8``), so the conv is taps (4, 4, 1) over 32 fp8 channels on the fp8 tile
    kernel; else None (the bf16 stem + a quantisation pass)."""
    N, D, H, W, C = in_shape5
    k = tuple(c1.kernel) if isinstance(c1.kernel, (tuple, list)) else (c1.kernel,) * 3
    st = tuple(c1.stride) if isinstance(c1.stride, (tuple, list)) else (c1.stride,) * 3
    if C != 1 or st != (2, 2, 2) or c1.padding != "valid" \
            or any(-(-kk // 2) != 4 for kk in k):
        return None
    OD, OH, OW = ((D - k[0]) // 2 + 1, (H - k[1]) // 2 + 1, (W - k[2]) // 2 + 1)
    D2, H2 = OD + 3, OH + 3                      # packed rows the 4 d / h taps reach
    if 2 * (D2 - 1) >= D or 2 * (H2 - 1) >= H or 2 * (OW - 1 + 3) >= W:
        return None
    spec = ConvSpec.make((N, D2, H2, OW, 32), c1.cout, (4, 4, 1), 1, "valid")
    if (spec.OD, spec.OH, spec.OW) != (OD, OH, OW):
        return None
    return spec


def stem_tap_weight(w: torch.Tensor) -> torch.Tensor:
    """[K, k, k, k, 1] stem weight -> [K, 4, 4, 1, 32]: space-to-depth weight [K, 4, 4, 4, 8]
    (tap 2t + p of each dim -> tap t, channel pd*4 + ph*2 + pw) with its w-taps folded into
    the channels (8 j + c)."""
    K = w.shape[0]
    wp = torch.zeros(K, 8, 8, 8, 1, dtype=torch.float32, device=w.device)
    wp[:, :w.shape[1], :w.shape[2], :w.shape[3]] = w.float()
    w2 = wp.view(K, 4, 2, 4, 2, 4, 2).permute(0, 1, 3, 5, 2, 4, 6).reshape(K, 4, 4, 4, 8)
    return w2.reshape(K, 4, 4, 1, 32).contiguous()


def stem_tap_input(x5: torch.Tensor, spec: ConvSpec, in_scale: float, int8: bool = False) -> torch.Tensor:
    """e4m3 (or int8) [N, D2, H2, OW, 32] tap-expanded space-to-depth input of the stem (one launch)."""
    N, D, H, W, _ = x5.shape
    x5 = x5.to(torch.bfloat16).contiguous()
    y = torch.empty(spec.N, spec.D, spec.H, spec.W, 32, dtype=torch.uint8, device=x5.device)
    _native.kernels().s2d_tap_f8(x5.data_ptr(), y.data_ptr(), [N, D, H, W, spec.D, spec.H, spec.W, 4], 1.0 / in_scale,
                                 _native.stream(x5), [x5.numel(), y.numel()], int(int8))
    return y


class Fp8FeatureNet3D:
    """Inference-only fp8 FeatureNet-3D built from a trained (or random-init) bf16 model.
    With a calibrated input scale, the stem runs in fp8 too (tap-expanded space-to-depth,
    :func:`stem_tap_plan`) and writes e4m3 straight into conv2's input."""

    def __init__(self, model: FeatureNet3D, act_scales: list[float], in_scale: float | None = None,
                 stem_int8: bool = False):
        self.model = model.eval()
        convs = list(model.convs)
        c1 = convs[0]
        w1, b1 = _fold_bn(c1)
        self.c1_w, self.c1_b = w1, b1
        self.act_scales = act_scales
        self.in_scale = in_scale
        self._stem_w2 = {}
        self._block_ok = {}
        self.calib_agreement = None
        # quantize_model(fallback=True): None (as built), "per_tensor" (block scales off for this
        # model) or "bf16" (the model itself); calib_history: (mode, agreement) per step tried
        self.fallback = None
        self.calib_history = []
        self.stem = None
        self.stem_int8 = bool(stem_int8)
        if in_scale is not None:
            self.stem = Fp8Conv(None, in_scale, act_scales[0], relu=True, wb=(stem_tap_weight(w1), b1),
                                padding="valid", int8=self.stem_int8)
        self.layers = []
        for i, conv in enumerate(convs[1:], start=1):
            last = i == len(convs) - 1
            self.layers.append(Fp8Conv(conv, act_scales[i - 1], None if last else act_scales[i], relu=True))
        self.pool = convs[-1].pool
        # the dense layers read bf16 weight copies
        self.fc_w = [fc.weight.detach().to(torch.bfloat16).contiguous() for fc in (model.fc1, model.fc2)]

    def _dense(self, f: torch.Tensor) -> torch.Tensor:
        m = self.model
        if self.fc_w is None or not _native.use_native(f):
            return m.fc2(m.fc1(f), out_fp32=True)
        from ..ops.linear import linear_infer
        h = linear_infer(f, self.fc_w[0], m.fc1.bias, m.fc1.act)
        return linear_infer(h, self.fc_w[1], m.fc2.bias, m.fc2.act, out_fp32=True)

    def block_mode(self, in_shape5: tuple) -> bool:
        """Block-scaled activations for this input: ``FN_F8_BLOCK`` on (default), the bf16 stem, and a
        block-scaled tile plan for every fp8 layer (else the per-tensor path)."""
        if os.environ.get("FN_F8_BLOCK", "1") == "0" or self.stem is not None or self.fallback is not None:
            return False
        key = (tuple(in_shape5), os.environ.get("FN_F8_TILE", "1"), os.environ.get("FN_F8_POOL", "1"))
        ok = self._block_ok.get(key)
        if ok is None:
            c1 = self.model.convs[0]
            shape = ConvSpec.make(key[0], c1.cout, c1.kernel, c1.stride, c1.padding).out_shape5
            ok = True
            for li, layer in enumerate(self.layers):
                spec = ConvSpec.make(shape, layer.K, layer.kernel, 1, layer.padding)
                last = li == len(self.layers) - 1
                tp = (layer.pool_plan(shape, block=True) if last and self._pool_fusable() else None) or \
                    layer.tile_plan(spec, block=True)
                if tp is None:
                    ok = False
                    break
                shape = spec.out_shape5 if not tp.pool else (spec.N, spec.OD // 2, spec.OH // 2, spec.OW // 2, spec.K)
            self._block_ok[key] = ok
        return ok

    @torch.no_grad()
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        m = self.model
        if x.dim() == 4:
            x = x.unsqueeze(-1)
        if self.fallback == "bf16":
            return m(x.to(torch.bfloat16)).float()
        c1 = m.convs[0]
        if self.block_mode(tuple(x.shape)):
            return self._forward_block(x)
        tspec = stem_tap_plan(c1, tuple(x.shape)) if self.stem is not None else None
        if tspec is not None and self.stem.tile_plan(tspec) is not None:
            xq, shape = self.stem(stem_tap_input(x, tspec, self.in_scale, self.stem_int8),   # fp8 / int8 in, fp8 out
                                  (tspec.N, tspec.D, tspec.H, tspec.W, tspec.C))
        else:
            # (uint8 voxels stay bytes: the space-to-depth packing reads them)
            x = x.contiguous() if x.dtype == torch.uint8 else x.to(torch.bfloat16).contiguous()
            spec = ConvSpec.make(tuple(x.shape), c1.cout, c1.kernel, c1.stride, c1.padding)
            xq = self._bf16_stem_fp8_out(x, spec)
            if xq is None:
                y = ops.conv(x, self.c1_w, self.c1_b, spec, "relu")           # bf16, BN folded, ReLU fused
                xq = quantize_fp8_act(y, self.act_scales[0])
            shape = spec.out_shape5
        fused_pool = False
        for li, layer in enumerate(self.layers):
            last = li == len(self.layers) - 1
            fused_pool = last and self._pool_fusable() and layer.pool_plan(shape) is not None
            xq, shape = layer(xq, shape, pool=fused_pool)
        feat = xq                                                             # bf16 [N, D, H, W, 64]
        if self.pool is not None and not fused_pool:
            ps = PoolSpec.make(tuple(feat.shape), self.pool, m.convs[-1].pool_stride, "valid")
            feat = ops.pool(feat, ps, "max")
        f = feat.reshape(feat.shape[0], -1)
        return self._dense(f)

    __call__ = forward

    def _forward_block(self, x: torch.Tensor) -> torch.Tensor:
        """Block-scaled fp8 forward: the bf16 stem writes (e4m3, scales) from its epilogue, every fp8
        layer reads them through the scaled MFMA and writes its own, the last one (fused pool) bf16."""
        m = self.model
        c1 = m.convs[0]
        x = x.contiguous() if x.dtype == torch.uint8 else x.to(torch.bfloat16).contiguous()
        spec = ConvSpec.make(tuple(x.shape), c1.cout, c1.kernel, c1.stride, c1.padding)
        xq = self._bf16_stem_fp8_out(x, spec, block=True)
        if xq is None:
            xq = quantize_fp8_block(ops.conv(x, self.c1_w, self.c1_b, spec, "relu"))
        shape = spec.out_shape5
        fused_pool = False
        for li, layer in enumerate(self.layers):
            last = li == len(self.layers) - 1
            fused_pool = last and self._pool_fusable() and layer.pool_plan(shape, block=True) is not None
            xq, shape = layer(xq, shape, pool=fused_pool)
        feat = xq
        if self.pool is not None and not fused_pool:
            ps = PoolSpec.make(tuple(feat.shape), self.pool, m.convs[-1].pool_stride, "valid")
            feat = ops.pool(feat, ps, "max")
        return self._dense(feat.reshape(feat.shape[0], -1))

    def _bf16_stem_fp8_out(self, x: torch.Tensor, spec: ConvSpec, block: bool = False):
        """The bf16 stem (space-to-depth tile kernel, BN folded, ReLU) writing e4m3 of its output
        / act_scales[0] from the epilogue -- conv2's input without a bf16 tensor or a
        quantisation pass -- or None where that kernel does not take the stem."""
        from ..ops.conv import s2d_input, s2d_plan, s2d_weight
        s2d = s2d_plan(spec)
        if s2d is None or os.environ.get("FN_F8_STEM_Q8", "1") == "0":
            return None
        f, spec2 = s2d
        tp = conv_tile.fwd_plan(spec2)
        if tp is None or tp.NT != 2 or tp.CS != 8:   # (the e4m3-output instances: 8-channel
            return None                                            #  slices, the space-to-depth stem)
        key = (f, spec2.C, spec2.KD, spec2.KH, spec2.KW)
        w2 = self._stem_w2.get(key)
        if w2 is None:
            w2 = self._stem_w2[key] = s2d_weight(self.c1_w, f, spec, spec2)
        x2 = s2d_input(x, f, spec2, (spec.pd, spec.ph, spec.pw))
        if block:                                # (block-scaled e4m3 + scale dwords)
            return conv_tile.conv_fwd_q8_block(x2, w2, self.c1_b, spec2, 1, tp)
        y, _ = conv_tile.conv_fwd(x2, w2, self.c1_b, spec2, 1, False, tp, out_scale=self.act_scales[0])
        return y

    def _pool_fusable(self) -> bool:
        """The model's max-pool is 2^3 with stride 2 ('valid'): the last conv's fp8 epilogue can
        pool (conv_tile pool plans)."""
        c = self.model.convs[-1]
        k = tuple(self.pool) if isinstance(self.pool, (tuple, list)) else (self.pool,) * 3
        st = c.pool_stride if getattr(c, "pool_stride", None) is not None else k
        st = tuple(st) if isinstance(st, (tuple, list)) else (st,) * 3
        return (self.pool is not None and k == (2, 2, 2) and st == (2, 2, 2) and c.pool_kind == "max"
                and c.pool_padding == "valid")


@torch.no_grad()
def calibrate(model: FeatureNet3D, calib_x: torch.Tensor, margin: float = 1.0) -> list[float]:
    """Per-layer post-ReLU activation scales (amax / 448) from a bf16 eval forward."""
    model.eval()
    x = calib_x
    if x.dim() == 4:
        x = x.unsqueeze(-1)
    x = x.to(torch.bfloat16)
    scales = []
    for conv in model.convs:
        x = conv(x)
        scales.append(max(float(x.float().abs().amax()) * margin, 1e-6) / FP8_MAX)
    return scales


def stem_mode() -> str:
    """FN_F8_STEM: '0' the bf16 stem writing e4m3 from its epilogue, '1' / 'e4m3' the stem on the
    fp8 kernel with per-channel e4m3 weights, 'i8' the stem on the int8 MFMA instance."""
    m = os.environ.get("FN_F8_STEM", "0")
    return {"1": "e4m3", "e4m3": "e4m3", "i8": "i8", "int8": "i8"}.get(m, "bf16")


CHECK_CHUNK = 64          # samples per forward of quantize_model's agreement check


def _agreement(model: FeatureNet3D, q: Fp8FeatureNet3D, x: torch.Tensor) -> float:
    """Top-1 agreement of the fp8 and bf16 models on ``x`` (in chunks of CHECK_CHUNK samples: two
    full-batch forwards over a 128^3 calibration set would double calibrate()'s peak activation
    memory)."""
    hits = 0
    with torch.no_grad():
        for i in range(0, x.shape[0], CHECK_CHUNK):
            xc = x[i:i + CHECK_CHUNK]
            a = model(xc.to(torch.bfloat16)).float().argmax(-1)
            b = q(xc).float().argmax(-1)
            hits += int((a == b).sum())
            del a, b
    return round(hits / max(1, x.shape[0]), 4)


def quantize_model(model: FeatureNet3D, calib_x: torch.Tensor, fp8_stem=None, fallback: bool = False,
                   fallback_at: float = FALLBACK_AT) -> Fp8FeatureNet3D:
    """fp8 model with activation scales from a bf16 pass over ``calib_x``.

    ``fp8_stem`` (default :func:`stem_mode`): 'bf16' keeps the stem on the bf16 tile kernel,
    writing e4m3 from its epilogue; 'e4m3' (or True) quantises the input too (scale amax / 448
    of the calibration input: binary voxels map exactly) and runs the stem on the fp8 kernel --
    per-channel e4m3 stem weights cost a trained model ~16 points of top-1 on the held-out set
    (the stem output error 6 % vs 3 %); 'i8' runs it on the int8 MFMA (v_mfma_i32_16x16x64_i8,
    2x the bf16 rate): binary inputs are exact in int8 and per-channel int8 weights keep ~8
    bits of each weight, the precision the e4m3 stem lacked.

    ``fallback``: the calibration check decides the numerics instead of only warning -- while the
    top-1 agreement with the bf16 model on ``calib_x`` is below ``fallback_at``, step down from
    block-scaled activations to per-tensor scales (the form that held the parity bar on the model
    where block scales did not, profiles/r5_fp8_block_parity.md), then to the bf16 model itself.
    ``q.fallback`` names the step taken, ``q.calib_history`` the agreement of each one tried.
    (Off by default: the kernel tests and the speed bench quantise random-init models, whose
    agreement says nothing about deployment.)"""
    if fp8_stem is None:
        fp8_stem = stem_mode()
    mode = {True: "e4m3", False: "bf16"}.get(fp8_stem, fp8_stem)
    if mode == "i8":
        from ..ops.conv_tile import experiments_built

        if not experiments_built():
            raise ValueError("the int8 fp8-stem instance is an experiment build (FN_BUILD_EXPERIMENTS=1): measured "
                             "no faster than the bf16 stem, and 23.8 points of top-1 lost on one of two seeds")
    amax = max(float(calib_x.float().abs().amax()), 1e-6)
    in_scale = {"e4m3": amax / FP8_MAX, "i8": amax / I8_MAX}.get(mode)
    q = Fp8FeatureNet3D(model, calibrate(model, calib_x), in_scale, stem_int8=mode == "i8")
    # post-quantisation check on the calibration set: top-1 agreement of the fp8 and bf16 models
    # (a model whose activations the chosen scales do not fit shows up here, not in deployment)
    x = calib_x if calib_x.dim() == 5 else calib_x.unsqueeze(-1)
    block = q.block_mode(tuple(x[:CHECK_CHUNK].shape))
    q.calib_agreement = _agreement(model, q, x)
    q.calib_history.append(("block" if block else "per_tensor", q.calib_agreement))
    if fallback and q.calib_agreement < fallback_at and block:
        q.fallback = "per_tensor"
        q.calib_agreement = _agreement(model, q, x)
        q.calib_history.append(("per_tensor", q.calib_agreement))
    if fallback and q.calib_agreement < fallback_at:
        q.fallback = "bf16"
        q.calib_agreement = 1.0
        q.calib_history.append(("bf16", 1.0))
    if q.calib_agreement < AGREEMENT_WARN:
        warnings.warn(f"fp8 model agrees with bf16 on {q.calib_agreement:.1%} of the calibration set "
                      f"(< {AGREEMENT_WARN:.0%}): keep this model in bf16", RuntimeWarning)
    return q


_ = math
