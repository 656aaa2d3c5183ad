"""Sub-pixel form of "nearest x2 upsample, then a 3^3 'same' conv" (the segmentation decoder).

    y(q) = sum_t W[t] . up(x)(q + t),   up(x)(q) = x(floor(q / 2)),   t in {-1, 0, 1}^3

Output position q = 2c + j (cell c on the low-resolution grid, parity j in {0, 1}^3) only
ever reads x at c + delta with delta in {j - 1, j} per dimension, so each of the 8 parity
classes is a 2^3-tap conv on x with its own folded weights

    Wf_j[e] = sum_t S[j][e][t] W[t],   S[j][e][t] = [floor((j + t) / 2) == j - 1 + e]

(8 taps instead of 27 per output: 3.4x fewer FLOPs, and up(x) is never materialised).

Backward works on the *shifted* space-to-depth view of dy: cell c' holds the
full-resolution positions q = 2c' - 1 + j' (j' in {0, 1}^3), 33^3 cells for a 64^3 grid,
256 channels (j', co) per cell, zero where q falls outside.  Then

  * dx(p) = sum_{e in {0,1}^3} sum_{j'} Kd[e][j']^T dy_sh(p + e, j'): one stride-1 2^3 'valid'
    conv over dy_sh, Kd[e][j'] = sum_t [0 <= 2e + j' + t - 1 <= 1] W[t];
  * dW = the adjoint of the weight fold above applied to the per-class weight gradients
    dWf_j[e] = sum_c dy(2c + j) (x) x(c + j - 1 + e).

This module holds the weight folds (tiny fp32 einsums, used on the GPU path too) and plain
PyTorch references of every piece for the CPU tests.  Reference parity: the decoder of
``FeatureNet3DSeg`` (SURVEY.md section 7.1 segmentation config), Keras ``UpSampling3D`` +
``Conv3D`` semantics (reference ``model/input.py:294`` for the conv).
"""
from __future__ import annotations

import itertools

import torch
import torch.nn.functional as F

PARITIES = list(itertools.product((0, 1), repeat=3))   # class index = (jd * 2 + jh) * 2 + jw


_SEL: dict = {}


def _cached(kind: str, make, device, dtype) -> torch.Tensor:
    """Selection matrices built on the host once per (device, dtype): a host-to-device copy
    (or an element store) is not allowed while a hipGraph is being captured, so the eager
    warmup steps create them and captured steps reuse them."""
    key = (kind, str(device), dtype)
    t = _SEL.get(key)
    if t is None:
        t = make().to(device=device, dtype=dtype)
        _SEL[key] = t
    return t


def _sel_fwd_cpu() -> torch.Tensor:
    s = torch.zeros(2, 2, 3)
    for j in range(2):
        for t in range(3):
            d = (j + t - 1) // 2                       # floor((j + tap) / 2), tap = t - 1
            s[j, d - (j - 1), t] = 1.0
    return s


def _sel_dgrad_cpu() -> torch.Tensor:
    s = torch.zeros(2, 2, 3)
    for e in range(2):
        for jp in range(2):
            for t in range(3):
                if 0 <= 2 * e + jp + (t - 1) - 1 <= 1:
                    s[e, jp, t] = 1.0
    return s


def _sel_fwd(device=None, dtype=torch.float32) -> torch.Tensor:
    """S[j][e][t] (1-D): parity j output, low-res offset j - 1 + e, full-res tap t - 1."""
    return _cached("fwd", _sel_fwd_cpu, device or "cpu", dtype)


def _sel_dgrad(device=None, dtype=torch.float32) -> torch.Tensor:
    """D[e][j'][t] (1-D): shifted cell p + e, sub-position j', full-res tap t - 1."""
    return _cached("dgrad", _sel_dgrad_cpu, device or "cpu", dtype)


def _wmap(src: torch.Tensor, K: int, C: int, mode: int, shape: tuple):
    """The native weight map (``conv_halo.hip`` subpixel_wmap) for fp32 GPU tensors, else None."""
    from .. import _native

    if not (src.is_cuda and src.dtype == torch.float32 and _native.kernels_available()):
        return None
    src = src.contiguous()
    out = torch.empty(shape, dtype=torch.float32, device=src.device)
    _native.kernels().subpixel_wmap(src.data_ptr(), out.data_ptr(), K, C, mode, _native.stream(src),
                                    [src.numel(), out.numel()])
    return out


def forward_weights(w: torch.Tensor) -> torch.Tensor:
    """W [K, 3, 3, 3, C] -> per-class folded weights [8, K, 2, 2, 2, C] (class = parity index)."""
    K, C = w.shape[0], w.shape[-1]
    out = _wmap(w, K, C, 0, (8, K, 2, 2, 2, C))
    if out is not None:
        return out
    s = _sel_fwd(w.device, w.dtype)
    # out[jd, jh, jw, k, ed, eh, ew, c]
    out = torch.einsum("adx,bey,cfz,kxyzi->abckdefi", s, s, s, w)
    return out.reshape(8, *out.shape[3:])


def fold_weight_grad(dwf: torch.Tensor) -> torch.Tensor:
    """Adjoint of :func:`forward_weights`: per-class [8, K, 2, 2, 2, C] -> dW [K, 3, 3, 3, C]."""
    K, C = dwf.shape[1], dwf.shape[-1]
    out = _wmap(dwf, K, C, 2, (K, 3, 3, 3, C))
    if out is not None:
        return out
    s = _sel_fwd(dwf.device, dwf.dtype)
    d = dwf.reshape(2, 2, 2, *dwf.shape[1:])
    return torch.einsum("adx,bey,cfz,abckdefi->kxyzi", s, s, s, d)


def dgrad_weights(w: torch.Tensor) -> torch.Tensor:
    """W [K, 3, 3, 3, C] -> the weights of the dgrad conv over the shifted view:
    [C (output), 2, 2, 2, 8 * K (input channel = j' * K + co)]."""
    K, C = w.shape[0], w.shape[-1]
    out = _wmap(w, K, C, 1, (C, 2, 2, 2, 8 * K))
    if out is not None:
        return out
    s = _sel_dgrad(w.device, w.dtype)
    # out[i, ed, eh, ew, jd, jh, jw, k]
    out = torch.einsum("dax,eby,fcz,kxyzi->idefabck", s, s, s, w)
    return out.reshape(C, 2, 2, 2, 8 * K)


def shift_s2d(dy: torch.Tensor) -> torch.Tensor:
    """Full-resolution [N, 2D, 2H, 2W, K] -> shifted space-to-depth [N, D+1, H+1, W+1, 8*K]
    (cell c' holds positions 2c' - 1 + j'; zero outside the grid).  Reference / CPU path."""
    N, FD, FH, FW, K = dy.shape
    p = F.pad(dy, (0, 0, 1, 1, 1, 1, 1, 1))               # [N, FD+2, FH+2, FW+2, K]
    D, H, W = FD // 2 + 1, FH // 2 + 1, FW // 2 + 1
    p = p.reshape(N, D, 2, H, 2, W, 2, K).permute(0, 1, 3, 5, 2, 4, 6, 7)
    return p.reshape(N, D, H, W, 8 * K)


def unshift_s2d(dsh: torch.Tensor, K: int) -> torch.Tensor:
    """Inverse of :func:`shift_s2d` (drops the zero border)."""
    N, D, H, W, _ = dsh.shape
    p = dsh.reshape(N, D, H, W, 2, 2, 2, K).permute(0, 1, 4, 2, 5, 3, 6, 7)
    p = p.reshape(N, 2 * D, 2 * H, 2 * W, K)
    return p[:, 1:-1, 1:-1, 1:-1].contiguous()


def _conv_cl(x: torch.Tensor, w: torch.Tensor, pad_lo: tuple, pad_hi: tuple) -> torch.Tensor:
    """Channels-last 'valid' conv3d after explicit (lo, hi) zero padding (fp32 reference)."""
    xp = F.pad(x, (0, 0, pad_lo[2], pad_hi[2], pad_lo[1], pad_hi[1], pad_lo[0], pad_hi[0]))
    y = F.conv3d(xp.permute(0, 4, 1, 2, 3), w.permute(0, 4, 1, 2, 3))
    return y.permute(0, 2, 3, 4, 1)


def class_pads(j: tuple) -> tuple[tuple, tuple]:
    """(lo, hi) zero padding of the low-res input for parity class j (offsets j - 1 + e)."""
    return tuple(1 - a for a in j), tuple(j)


def ref_forward(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """y = conv3^3_same(upsample2x(x)) through the 8 parity classes (fp32 reference)."""
    N, D, H, W, _ = x.shape
    wf = forward_weights(w)
    y = x.new_zeros(N, 2 * D, 2 * H, 2 * W, w.shape[0])
    for ci, j in enumerate(PARITIES):
        lo, hi = class_pads(j)
        y[:, j[0]::2, j[1]::2, j[2]::2] = _conv_cl(x, wf[ci], lo, hi)
    return y


def ref_dgrad(dy: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """dx of :func:`ref_forward` as the stride-1 2^3 conv over the shifted view (fp32 reference)."""
    return _conv_cl(shift_s2d(dy), dgrad_weights(w), (0, 0, 0), (0, 0, 0))


def ref_wgrad_classes(dy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """Per-class weight gradients [8, K, 2, 2, 2, C] (fp32 reference of the sub-pixel wgrad)."""
    K, C = dy.shape[-1], x.shape[-1]
    out = []
    for j in PARITIES:
        lo, hi = class_pads(j)
        xp = F.pad(x, (0, 0, lo[2], hi[2], lo[1], hi[1], lo[0], hi[0]))
        dyj = dy[:, j[0]::2, j[1]::2, j[2]::2]
        # dWf[k, e, c] = sum_{n, cell} dyj[n, cell, k] * xp[n, cell + e, c]
        g = torch.zeros(K, 2, 2, 2, C, dtype=dy.dtype, device=dy.device)
        D, H, W = dyj.shape[1:4]
        for ed, eh, ew in itertools.product(range(2), repeat=3):
            xs = xp[:, ed:ed + D, eh:eh + H, ew:ew + W]
            g[:, ed, eh, ew] = torch.einsum("ndhwk,ndhwc->kc", dyj, xs)
        out.append(g)
    return torch.stack(out)


# ---------------------------------------------------------------------------
# GPU path: decoder conv + BN + ReLU + 1x1 head as one autograd node
# ---------------------------------------------------------------------------
def gpu_ok(x5: torch.Tensor, K: int, C: int) -> bool:
    """The native sub-pixel path applies: bf16 GPU input, Cout 32 per class, C % 32 == 0."""
    import os

    from .. import _native
    from . import conv_tile, conv_wtile

    if os.environ.get("FN_SUBPIXEL", "1") == "0" or not _native.use_native(x5) or not conv_tile.enabled():
        return False
    N, D, H, W, Cx = x5.shape
    return (Cx == C and K == 32 and C % 32 == 0 and conv_tile.plan(N, (D, H, W), (2, 2, 2), C, K) is not None
            and _dgrad_plan(x5.shape, K) is not None
            and conv_wtile.plan_subpixel(N, (D, H, W), C, K) is not None)


def upconv_forward(x5: torch.Tensor, w: torch.Tensor):
    """y = conv3^3_same(upsample2x(x)) [N, 2D, 2H, 2W, K] bf16 + its BN statistics slab, as 8
    parity-class 2^3 convs on the tile kernel writing straight into the full-res output."""
    from . import conv_tile

    import dataclasses

    N, D, H, W, C = x5.shape
    K = w.shape[0]
    p = conv_tile.plan(N, (D, H, W), (2, 2, 2), C, K)
    # the 8 classes' weights as ONE packed stream of 8 K columns (one pack launch, not eight): class
    # ci's columns are fragment block ci of every k-step row, so its conv reads the stream from
    # fragment ci * nct on with the row pitch of all 8 (geometry nct = 8 nct)
    p8 = dataclasses.replace(p, nct=8 * p.nct)
    wf = forward_weights(w.detach().float()).reshape(8 * K, 8, C)
    wall = conv_tile.pack_weights(wf, 8 * K, 8, C, p8, dgrad=False)
    y = torch.empty(N, 2 * D, 2 * H, 2 * W, K, dtype=torch.bfloat16, device=x5.device)
    geoms = []
    for j in PARITIES:
        lo, _ = class_pads(j)
        geoms.append(conv_tile.geometry(p8, (N, D, H, W, C), (D, H, W), (2, 2, 2), lo,
                                        view=conv_tile.parity_view((2 * D, 2 * H, 2 * W), j)))
    nw = conv_tile.workers(p8, geoms[0], K)
    slab = torch.empty(8 * nw, 2, K, dtype=torch.float32, device=x5.device)
    frag = 64 * 8                                # bf16 elements per packed fragment
    for ci in range(8):
        conv_tile.run(x5, wall[ci * p.nct * frag:], None, y, slab[ci * nw:(ci + 1) * nw], p8, geoms[ci], (2, 2, 2), K,
                      0)
    return y, slab


def _dgrad_plan(x_shape, K: int, nt4: bool = True):
    """The dgrad's tile plan: 8 taps over the 8K shifted-layout channels into C columns -- DMA-bound
    (each job's halo feeds only 8 taps), so C = 64 takes 64-column workgroups (one halo DMA for
    all the columns instead of one per 32-column block: 1.70 -> 1.50 ms at batch 128, seg step
    -1.4 %, profiles/r6_subpixel_nt4.md)."""
    from . import conv_tile

    N, D, H, W, C = x_shape
    return (nt4 and conv_tile.plan(N, (D, H, W), (2, 2, 2), 8 * K, C, nt4=True)) or \
        conv_tile.plan(N, (D, H, W), (2, 2, 2), 8 * K, C)


def upconv_dgrad(dsh: torch.Tensor, w: torch.Tensor, x_shape, mask=None, nt4: bool = True):
    """dx [N, D, H, W, C] = the 2^3 'valid' conv over the shifted view with :func:`dgrad_weights`.
    ``mask`` (x = relu(bn(y)) with its relu-mask bytes, the BN statistics identity of
    ops/bnfuse.py): returns ``(dx, slab)``, the slab's row 0 the column sums of dx * relu'(x)."""
    from . import conv_tile

    N, D, H, W, C = x_shape
    K = w.shape[0]
    p = _dgrad_plan(x_shape, K, nt4)
    kd = dgrad_weights(w.detach().float()).reshape(C, 8, 8 * K)
    wpk = conv_tile.pack_weights(kd, C, 8, 8 * K, p, dgrad=False)
    geom = conv_tile.geometry(p, (N, D + 1, H + 1, W + 1, 8 * K), (D, H, W), (2, 2, 2), (0, 0, 0))
    dx = torch.empty(N, D, H, W, C, dtype=torch.bfloat16, device=dsh.device)
    if mask is None:
        conv_tile.run(dsh, wpk, None, dx, None, p, geom, (2, 2, 2), C, 0)
        return dx
    assert mask.numel() * 8 == dx.numel() and mask.dtype == torch.uint8
    slab = torch.empty(conv_tile.workers(p, geom, C), 2, C, dtype=torch.float32, device=dsh.device)
    conv_tile.run(dsh, wpk, None, dx, slab, p, geom, (2, 2, 2), C, 0, bny=mask)
    return dx, slab


def _bn_source(ctx, x: torch.Tensor, K: int) -> None:
    """Forward: when the decoder's input is a tagged relu(bn(y)) with its relu mask (the
    encoder's last BN, ops/bnfuse.py) and the dgrad plan takes the mask epilogue, keep the
    source for the backward's statistics identity."""
    from . import bnfuse, conv_tile

    ctx.bn_src = None
    if not ctx.needs_input_grad[0]:
        return
    src = bnfuse.source_of(x)
    if src is None or src[3] is None or src[2] != 1:
        return
    p = _dgrad_plan(tuple(x.shape), K)
    if p is not None and conv_tile.mask_dgrad_ok(p, x.shape[-1]):
        ctx.bn_src = src


def _decoder_backward(ctx, dsh: torch.Tensor, w: torch.Tensor, x: torch.Tensor, K: int):
    """(dx, dw) of the sub-pixel decoder conv from the shifted dy; with a BN source
    (:func:`_bn_source`) the dgrad sums that BN's g = dx * relu' and, once the class weight
    gradients exist, S = sum W_class . dW_class (the adjoint identity holds class by class: the
    dgrad's weights are the class weights re-indexed) goes to the BN backward with it."""
    from . import bnfuse, conv_wtile
    from .conv import bn_wdot

    src, ctx.bn_src = getattr(ctx, "bn_src", None), None
    dx = slab = None
    if ctx.needs_input_grad[0]:
        if src is not None:
            dx, slab = upconv_dgrad(dsh, w, x.shape, mask=src[3])
        else:
            dx = upconv_dgrad(dsh, w, x.shape)
    dw = None
    if ctx.needs_input_grad[1]:
        N, D, H, W, C = x.shape
        p = conv_wtile.plan_subpixel(N, (D, H, W), C, K)
        dwf = conv_wtile.conv_wgrad_subpixel(dsh, x, p)
        if slab is not None:
            wf = forward_weights(w.detach().float()).reshape(-1, C).contiguous()
            bnfuse.offer(dx, ("identity", slab, bn_wdot(wf, dwf.reshape(-1, C), None)), src[0])
        dw = fold_weight_grad(dwf).reshape(w.shape)
    return dx, dw


def bn_bwd_to_shifted(dz2, y2, prm, dbeta, dgamma, act: int, full_shape) -> torch.Tensor:
    """BN(+act) backward of the decoder output, written as the shifted space-to-depth dy."""
    from .. import _native

    N, FD, FH, FW, K = full_shape
    dsh = torch.empty(N, FD // 2 + 1, FH // 2 + 1, FW // 2 + 1, 8 * K, dtype=torch.bfloat16, device=y2.device)
    _native.kernels().bn_bwd_apply_s2d(dz2.data_ptr(), y2.data_ptr(), prm[2].data_ptr(), prm[3].data_ptr(),
                                       prm[0].data_ptr(), prm[1].data_ptr(), dbeta.data_ptr(), dgamma.data_ptr(),
                                       dsh.data_ptr(), N, FD, FH, FW, K, 1.0 / y2.shape[0], act,
                                       _native.stream(y2), [y2.numel(), dsh.numel()])
    return dsh


def _head_forward(x, w, gamma, beta, rmean, rvar, momentum, eps, hw, hb):
    """Decoder forward up to the head's input: (y, its BN parameters, head weight [NC, K], bias)."""
    from . import bn as bn_ops

    y, slab = upconv_forward(x, w)
    K = y.shape[-1]
    prm = bn_ops._finalize_fwd(slab, y.numel() // K, gamma, beta, rmean, rvar, momentum, eps)
    w2 = hw.detach().reshape(hw.shape[0], K)
    bias = hb.detach().float().contiguous() if hb is not None else None
    return y, prm, w2, bias


def _head_backward(ctx, d2):
    """Backward of decoder + head from d(logits) d2 [M, NC] (bf16): the input and parameter
    gradients in SubpixelDecoderHeadFn.backward's order."""
    from .. import _native
    from . import bn as bn_ops
    from ..training.flat import grad_target
    from .conv import native_colsum, pw_wgrad

    x, w, y, prm, hw = ctx.saved_tensors
    K = y.shape[-1]
    NC = hw.shape[0]
    y2 = y.reshape(-1, K)
    w2 = hw.detach().reshape(NC, K)
    dhw = (pw_wgrad(d2, y2, pro=(prm[2], prm[3], ctx.act), out=grad_target(hw)).reshape(hw.shape)
           if ctx.needs_input_grad[9] else None)
    dhb = native_colsum(d2, out=grad_target(ctx.bparam)) if (ctx.has_b and ctx.needs_input_grad[10]) else None
    M = y2.shape[0]
    Kn = _native.kernels()
    part = torch.empty(Kn.pw_fwd_blocks(M, NC, K), 2, K, dtype=torch.float32, device=y.device)
    dz2 = torch.empty(M, K, dtype=torch.bfloat16, device=y.device)
    wb = w2.t().to(torch.bfloat16).contiguous()
    Kn.pw_fwd(d2.data_ptr(), wb.data_ptr(), 0, dz2.data_ptr(), M, NC, K, 0, _native.stream(d2), 0, 0, 0,
              y2.data_ptr(), prm[2].data_ptr(), prm[3].data_ptr(), part.data_ptr(), ctx.act)
    dbeta, dgamma = bn_ops._bwd_param_grads(dz2, y2, prm, ctx.act, *ctx.params, part=part)
    dsh = bn_bwd_to_shifted(dz2, y2, prm, dbeta, dgamma, ctx.act, y.shape)
    dx, dw = _decoder_backward(ctx, dsh, w, x, K)
    return (dx, dw, dgamma if ctx.needs_input_grad[2] else None, dbeta if ctx.needs_input_grad[3] else None,
            None, None, None, None, None, dhw, dhb)


class SubpixelDecoderHeadFn(torch.autograd.Function):
    """logits = head(relu(bn(conv3^3_same(upsample2x(x))))) without materialising upsample2x(x)
    or relu(bn(.)) (FeatureNet3DSeg's decoder + 1x1 head, training mode).

    Forward: 8 parity-class convs (tile kernel, strided output view) + BN statistics from
    their epilogues, then the pointwise head with the BN + ReLU prologue (as
    ``ops.bn.BatchNormActPointwiseFn``).  Backward: head dgrad (+ this BN's backward
    moments), head wgrad, BN backward written as the shifted space-to-depth dy, then the
    decoder dgrad (one 2^3 conv over it) and weight gradient (the sub-pixel conv_wtile form +
    the adjoint weight fold)."""

    @staticmethod
    def forward(ctx, x, w, gamma, beta, rmean, rvar, momentum, eps, act, hw, hb):
        from .conv import pw_fwd

        y, prm, w2, bias = _head_forward(x, w, gamma, beta, rmean, rvar, momentum, eps, hw, hb)
        _bn_source(ctx, x, w.shape[0])
        out = pw_fwd(y.reshape(-1, y.shape[-1]), w2, bias, 0, pro=(prm[2], prm[3], act))
        ctx.save_for_backward(x, w, y, prm, hw)
        ctx.act, ctx.has_b, ctx.bparam = act, hb is not None, hb
        ctx.params = (beta, gamma)
        return out.reshape(*y.shape[:-1], hw.shape[0])

    @staticmethod
    def backward(ctx, dout):
        return _head_backward(ctx, dout.contiguous().to(torch.bfloat16).reshape(-1, ctx.saved_tensors[4].shape[0]))


class SubpixelDecoderHeadXentFn(torch.autograd.Function):
    """(mean softmax cross-entropy, top-1 hits) of the per-voxel logits of
    :class:`SubpixelDecoderHeadFn` against int64 ``labels`` -- with the loss in the head's
    epilogue (``pw_fwd_kernel`` XENT instance): the forward stores d(loss)/d(logits) instead of
    the 838M logits of a 128 x 64^3 batch, and the separate loss kernel disappears (reference:
    the softmax head + categorical cross-entropy, ``model/keras_model.py:124``,
    ``tensorflow_generator.py:232-235``)."""

    @staticmethod
    def forward(ctx, x, w, gamma, beta, rmean, rvar, momentum, eps, act, hw, hb, labels, smoothing, want_hits=True):
        from .. import _native

        y, prm, w2, bias = _head_forward(x, w, gamma, beta, rmean, rvar, momentum, eps, hw, hb)
        _bn_source(ctx, x, w.shape[0])
        K = y.shape[-1]
        y2 = y.reshape(-1, K)
        M, NC = y2.shape[0], w2.shape[0]
        Kn = _native.kernels()
        lab = labels.reshape(-1).contiguous()
        dlog = torch.empty(M, NC, dtype=torch.bfloat16, device=y.device)
        xpart = torch.empty(Kn.pw_xent_blocks(M), 2, dtype=torch.float32, device=y.device)
        wb = w2.to(torch.bfloat16).contiguous()
        Kn.pw_fwd_xent(y2.data_ptr(), wb.data_ptr(), _native.ptr(bias), dlog.data_ptr(), M, K, NC,
                       prm[2].data_ptr(), prm[3].data_ptr(), act, lab.data_ptr(), xpart.data_ptr(), 1.0 / M,
                       float(smoothing), _native.stream(y2), [y2.numel(), dlog.numel(), lab.numel(), xpart.numel()])
        ctx.save_for_backward(x, w, y, prm, hw, dlog)
        ctx.act, ctx.has_b, ctx.bparam = act, hb is not None, hb
        ctx.params = (beta, gamma)
        hits = xpart[:, 1].double().sum().round().long()   # (fp64: > 2^24 voxels per batch)
        ctx.mark_non_differentiable(hits)
        return xpart[:, 0].sum() / M, hits

    @staticmethod
    def backward(ctx, dloss, _dhits):
        from .. import _native

        dlog = ctx.saved_tensors[5]
        # d(logits) carries 1/M; scale by dloss in place -- a near-empty launch when dloss == 1
        from .loss import is_unit

        if not is_unit(dloss):                   # (the unit seed: nothing to scale)
            s = dloss.detach().float().reshape(1).contiguous()
            _native.kernels().scale_unless_one(dlog.data_ptr(), 1, s.data_ptr(), dlog.numel(), _native.stream(dlog))
        g = _head_backward(_SavedView(ctx), dlog)
        return g + (None, None)


class SubpixelDecoderHeadLossFn(torch.autograd.Function):
    """(mean softmax cross-entropy, top-1 hits) of FeatureNet3DSeg's decoder + head with the
    head's ENTIRE backward done in the forward pass (``csrc/kernels/seghead.hip``): one
    streaming kernel computes logits, loss, d(logits), the head weight / bias gradient partials,
    dz = d(logits) W and the decoder BN's backward moments while each 256-voxel tile is in LDS,
    and writes only dz.  The backward sums the partials, scales by dloss (a near-empty launch
    when it is 1) and continues with the BN backward and the decoder.  K = 32 decoder channels,
    NC <= 32 classes."""

    @staticmethod
    def forward(ctx, x, w, gamma, beta, rmean, rvar, momentum, eps, act, hw, hb, labels, smoothing, want_hits=True):
        from .. import _native

        y, prm, w2, bias = _head_forward(x, w, gamma, beta, rmean, rvar, momentum, eps, hw, hb)
        _bn_source(ctx, x, w.shape[0])
        K = y.shape[-1]
        y2 = y.reshape(-1, K)
        M, NC = y2.shape[0], w2.shape[0]
        Kn = _native.kernels()
        lab = labels.reshape(-1).contiguous()
        dz = torch.empty(M, K, dtype=torch.bfloat16, device=y.device)
        nb = Kn.seghead_blocks(M)
        part = torch.empty(nb, Kn.seghead_part_len(), dtype=torch.float32, device=y.device)
        wb = w2.to(torch.bfloat16).contiguous()
        Kn.seghead_loss(y2.data_ptr(), prm[2].data_ptr(), prm[3].data_ptr(), wb.data_ptr(), _native.ptr(bias),
                        lab.data_ptr(), dz.data_ptr(), part.data_ptr(), M, K, NC, act, 1.0 / M, float(smoothing),
                        _native.stream(y2), [y2.numel(), wb.numel(), lab.numel(), dz.numel(), part.numel()],
                        int(lab.dtype == torch.uint8), int(bool(want_hits)))
        # the workgroups' partials summed once, in row order (one launch), for the loss here and the
        # head / BN-moment gradients in the backward
        tot = torch.empty(part.shape[1], dtype=torch.float32, device=y.device)
        Kn.part_reduce(part.data_ptr(), tot.data_ptr(), part.shape[1], part.shape[0], 0, _native.stream(y2),
                       [part.numel(), tot.numel()])
        ctx.save_for_backward(x, w, y, prm, hw, dz, tot)
        ctx.act, ctx.has_b, ctx.bparam = act, hb is not None, hb
        ctx.params = (beta, gamma)
        # top-1 hits only when asked for (fp64: > 2^24 voxels per batch; four small launches)
        hits = part[:, 1].double().sum().round().long() if want_hits else torch.empty(0, dtype=torch.long,
                                                                                        device=y.device)
        ctx.mark_non_differentiable(hits)
        return tot[0] / M, hits

    @staticmethod
    def backward(ctx, dloss, _dhits):
        from .. import _native
        from . import bn as bn_ops
        from ..training.flat import grad_target

        x, w, y, prm, hw, dz, tot = ctx.saved_tensors
        K = y.shape[-1]
        NC = hw.shape[0]
        y2 = y.reshape(-1, K)
        from .loss import is_unit

        s = dloss.detach().float().reshape(1).contiguous()
        if not is_unit(dloss):
            _native.kernels().scale_unless_one(dz.data_ptr(), 1, s.data_ptr(), dz.numel(), _native.stream(dz))
        tot = tot[2:] if is_unit(dloss) else tot[2:] * s   # [db 32 | dWt 32 x 32 | msum 32 | msq 32], x dloss
        dhw = dhb = None
        if ctx.needs_input_grad[9]:
            dwt = tot[32:32 + 32 * 32].view(32, 32)[:K, :NC]    # [ch][cls]
            tgt = grad_target(hw)
            dhw = tgt.view(NC, K).copy_(dwt.t()) if tgt is not None else dwt.t().contiguous()
            dhw = dhw.reshape(hw.shape)
        if ctx.has_b and ctx.needs_input_grad[10]:
            tgt = grad_target(ctx.bparam)
            dhb = tgt.copy_(tot[:NC]) if tgt is not None else tot[:NC].clone()
        mom = tot[32 + 32 * 32:].view(1, 2, 32)[:, :, :K].contiguous()   # (sum g, sum g*y) of the BN
        dbeta, dgamma = bn_ops._bwd_param_grads(dz, y2, prm, ctx.act, *ctx.params, part=mom)
        dsh = bn_bwd_to_shifted(dz, y2, prm, dbeta, dgamma, ctx.act, y.shape)
        dx, dw = _decoder_backward(ctx, dsh, w, x, K)
        return (dx, dw, dgamma if ctx.needs_input_grad[2] else None, dbeta if ctx.needs_input_grad[3] else None,
                None, None, None, None, None, dhw, dhb, None, None, None)


class _SavedView:
    """ctx stand-in for :func:`_head_backward` (its first five saved tensors, the same flags)."""

    def __init__(self, ctx):
        self.saved_tensors = ctx.saved_tensors[:5]
        self.needs_input_grad = ctx.needs_input_grad
        self.act, self.has_b, self.bparam, self.params = ctx.act, ctx.has_b, ctx.bparam, ctx.params
        self.bn_src, ctx.bn_src = getattr(ctx, "bn_src", None), None


def decoder_head(x5, w, gamma, beta, running_mean, running_var, hw, hb, momentum=0.1, eps=1e-5, act="relu"):
    """Training-mode decoder (upsample x2 + 3^3 conv + BN + act) + 1x1 head on the sub-pixel
    GPU path (caller checks :func:`gpu_ok`)."""
    from .spec import act_code

    return SubpixelDecoderHeadFn.apply(x5.to(torch.bfloat16).contiguous(), w, gamma, beta, running_mean,
                                       running_var, momentum, eps, act_code(act), hw, hb)


def decoder_head_xent(x5, w, gamma, beta, running_mean, running_var, hw, hb, labels, momentum=0.1, eps=1e-5,
                      act="relu", smoothing: float = 0.0, want_hits: bool = True):
    """:func:`decoder_head` + mean softmax cross-entropy against per-voxel ``labels`` -> (loss, hits)
    (caller checks :func:`gpu_ok` and :func:`xent_ok`): the head's whole backward inside the
    forward kernel (:class:`SubpixelDecoderHeadLossFn`) for 32 decoder channels
    (``FN_SEG_XENT=2`` keeps the loss-only epilogue, :class:`SubpixelDecoderHeadXentFn`)."""
    import os

    from .spec import act_code

    if hw.shape[-1] == 32 and os.environ.get("FN_SEG_XENT", "1") != "2":
        # (uint8 labels stay uint8: the kernel reads either, a byte is 8x fewer label bytes)
        lab = labels if labels.dtype == torch.uint8 else labels.long()
        return SubpixelDecoderHeadLossFn.apply(x5.to(torch.bfloat16).contiguous(), w, gamma, beta, running_mean,
                                               running_var, momentum, eps, act_code(act), hw, hb, lab,
                                               float(smoothing), bool(want_hits))
    return SubpixelDecoderHeadXentFn.apply(x5.to(torch.bfloat16).contiguous(), w, gamma, beta, running_mean,
                                           running_var, momentum, eps, act_code(act), hw, hb, labels.long(),
                                           float(smoothing))


def xent_ok(K: int, NC: int) -> bool:
    """Shapes the fused head + loss kernel takes (K, NC <= 32; FN_SEG_XENT=0 turns it off)."""
    import os

    return os.environ.get("FN_SEG_XENT", "1") != "0" and K <= 32 and 2 <= NC <= 32
