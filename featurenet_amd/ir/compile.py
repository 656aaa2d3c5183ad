"""Lower a :class:`~featurenet_amd.ir.spec.ModelSpec` to a trainable module.

This is the framework's graph builder, replacing the reference's Keras graph
construction (``KerasFeatureModel.build``, ``model/keras_model.py:105-159``;
``Block.build_tensorflow_model``, ``model/block.py:48-77``;
``Cell.build_tensorflow_model``, ``model/cell.py:47-86``).  Construction runs
on *symbolic shapes* first (no tensors), creating native-op modules and a flat
program; ``CandidateNet.forward`` then executes the program.  The reference's
routing semantics are reproduced exactly:

* the block input stack starts as ``[X]``; a cell reads the stack entries that
  are raw tensors or cell outputs whose countdown reached 0 -- ``input1``
  takes the first, ``input2`` the second (else the first);
* block stride / feature multiplier are pushed into both inputs (stride
  clamped to [1, 2], features = in_channels x multiplier clamped to [6, 2048]);
* ``input2 == Zeros`` short-circuits the second branch;
* ``OutCell(r)`` is pushed to the front of the stack with countdown ``r+1``
  (the ``min(max_relative_index, .)`` clamp is overwritten by ``OutCell.build``
  in the reference and therefore has no effect); every cell end decrements
  pending countdowns; ``Out`` appends to the model outputs; ``OutBlock`` is
  dropped;
* block exit forwards ``[stack head, block input]`` (the reference's
  ``i is OutBlock`` instance-vs-class test is always false);
* head: last ``Out`` or the stack head, flattened, then ``Dense(n_classes)``
  (softmax fused into the loss);
* channel harmonisation of 4-D branches (1x1 conv on the wider branch with
  stride = int(W ratio)), ``Sum``/``Concat`` fall back to branch 2 on shape
  mismatch, ``Concat`` and ``BatchNormalization`` act on axis 1 (``compat=True``;
  ``compat=False`` uses the channel axis instead);
* models above 20M parameters are rejected (``keras_model.py:127-130``).

Any construction error marks the candidate invalid (``CompileError``), the
reference's "build returns None" semantics.
"""
from __future__ import annotations

import importlib
import math
from dataclasses import dataclass

import torch
from torch import nn

from .. import ops
from ..models.layers import AxisBatchNorm, Conv, Dense, DepthwiseConv, Pool, SeparableConv
from .spec import CellSpec, InputSpec, ModelSpec, OpSpec

conv_ops = importlib.import_module("..ops.conv", __package__)   # (the module: ops.conv is the conv function)

MIN_FEATURES, MAX_FEATURES = 6, 2048
MAX_PARAMS = 20_000_000


class CompileError(Exception):
    pass


class ModelTooLarge(CompileError):
    pass


@dataclass
class Sym:
    node: int
    shape: tuple            # without the batch dimension

    @property
    def rank(self) -> int:  # Keras ndims (with batch)
        return len(self.shape) + 1


@dataclass
class _Entry:
    kind: str               # raw | cell | block
    sym: Sym
    current: int = 0


class _Builder:
    def __init__(self, input_shape: tuple, compat: bool, fill_defaults: bool = False):
        self.compat = compat
        self.fill_defaults = fill_defaults
        self.mods = nn.ModuleList()
        self.prog: list[tuple] = []
        self.cost: list[tuple] = []     # per instruction: (params, flops, keras layers)
        self.params = 0
        self.flops = 0
        self.layers = 1  # the Input layer
        self.x = self._emit(("input", None, ()), tuple(input_shape))

    def _emit(self, instr: tuple, shape: tuple, cost: tuple = (0, 0, 0)) -> Sym:
        self.prog.append(instr)
        self.cost.append(cost)
        return Sym(len(self.prog) - 1, tuple(int(s) for s in shape))

    def module(self, mod: nn.Module, x: Sym, shape: tuple, flops: int = 0) -> Sym:
        self.mods.append(mod)
        n = sum(p.numel() for p in mod.parameters()) + sum(b.numel() for b in mod.buffers())
        self.params += n
        self.flops += flops
        self.layers += 1
        return self._emit(("module", len(self.mods) - 1, (x.node,)), shape, (n, flops, 1))

    def fn(self, name: str, args, ins: tuple, shape: tuple, layer: bool = True) -> Sym:
        if layer:
            self.layers += 1
        return self._emit((name, args, tuple(s.node for s in ins)), shape, (0, 0, int(layer)))

    def prune(self, out: int) -> None:
        """Dead-code elimination: keep only instructions the output depends on.

        A Keras functional ``Model(inputs, outputs)`` only contains layers reachable
        from its outputs, so cells whose results the block/OutCell wiring drops
        (``model/block.py``, ``model/cell.py``) neither count towards
        ``count_params`` nor run; the same holds here.
        """
        live = [False] * len(self.prog)
        live[out] = True
        live[0] = True
        for i in range(out, -1, -1):
            if live[i]:
                for j in self.prog[i][2]:
                    live[j] = True
        remap, prog, cost, mods, mremap = {}, [], [], nn.ModuleList(), {}
        for i, (kind, arg, ins) in enumerate(self.prog[:out + 1]):
            if not live[i]:
                continue
            if kind in ("module", "head"):
                if arg not in mremap:
                    mremap[arg] = len(mods)
                    mods.append(self.mods[arg])
                arg = mremap[arg]
            remap[i] = len(prog)
            prog.append((kind, arg, tuple(remap[j] for j in ins)))
            cost.append(self.cost[i])
        self.prog, self.cost, self.mods = prog, cost, mods
        self.params = sum(c[0] for c in cost)
        self.flops = sum(c[1] for c in cost)
        self.layers = 1 + sum(c[2] for c in cost)
        self.fold_pads()

    def fold_pads(self) -> None:
        """ZeroPadding2D whose only consumer is a convolution: the convolution takes the
        padding into its own (zero) border instead and the pad becomes an alias of its input
        -- no padded tensor is materialised.  The instruction stays (Keras counts the
        ZeroPadding layer in ``nb_layers``)."""
        from ..models.layers import Conv

        users: dict = {}
        for j, (kind, arg, ins) in enumerate(self.prog):
            for i in ins:
                users.setdefault(i, []).append(j)
        for i, (kind, arg, ins) in enumerate(self.prog):
            if kind != "pad" or len(users.get(i, [])) != 1:
                continue
            j = users[i][0]
            jk, ja, jins = self.prog[j]
            if jk != "module" or jins != (i,) or not isinstance(self.mods[ja], Conv):
                continue
            conv = self.mods[ja]
            if getattr(conv, "extra_pad", (0, 0, 0)) != (0, 0, 0):
                continue
            ph, pw = arg
            if not _pad_foldable(conv, (0, ph, pw)):
                continue
            conv.extra_pad = (0, ph, pw)
            self.prog[i] = ("alias", None, ins)

    # ----------------------------------------------------------------- layers
    def conv(self, x: Sym, features: int, kernel, stride, padding: str, act, ctype: str) -> Sym:
        spatial = x.shape[:-1]
        nd = len(spatial)
        C = x.shape[-1]
        k = _fit(kernel, nd)
        s = _fit(stride or 1, nd)
        pad = "same" if padding not in ("valid",) else "valid"
        out_sp = tuple(_conv_out(i, kk, ss, pad) for i, kk, ss in zip(spatial, k, s))
        if min(out_sp) <= 0:
            raise CompileError(f"conv kernel {k} larger than input {spatial} with valid padding")
        kfull, sfull = _pad3(k, 1), _pad3(s, 1)
        fused_act = act if act in (None, "relu", "tanh", "sigmoid") else None
        vox = math.prod(out_sp)
        if ctype == "normal":
            mod = Conv(C, features, kfull, sfull, pad, act=fused_act, bias=True)
            y = self.module(mod, x, out_sp + (features,), 2 * vox * features * C * math.prod(k))
        elif ctype == "separable":
            mod = SeparableConv(C, features, kfull, sfull, pad, act=fused_act)
            y = self.module(mod, x, out_sp + (features,), 2 * vox * (C * math.prod(k) + C * features))
        elif ctype == "depthwise":
            mod = DepthwiseConv(C, kfull, sfull, pad, act=fused_act)
            y = self.module(mod, x, out_sp + (C,), 2 * vox * C * math.prod(k))
        else:
            return x
        if act not in (None, "relu", "tanh", "sigmoid"):
            y = self.fn("act", act, (y,), y.shape, layer=False)
        return y

    def pool(self, x: Sym, kernel, stride, ptype: str, padding: str) -> Sym:
        spatial = x.shape[:-1]
        nd = len(spatial)
        C = x.shape[-1]
        if ptype == "global":
            return self.fn("gap", None, (x,), (C,))
        k = _fit(kernel, nd)
        s = _fit(stride or 1, nd)
        pad = "same" if padding != "valid" else "valid"
        out_sp = tuple(_conv_out(i, kk, ss, pad) for i, kk, ss in zip(spatial, k, s))
        if min(out_sp) <= 0:
            raise CompileError("pooling window larger than input")
        mod = Pool(_pad3(k, 1), _pad3(s, 1), pad, "max" if ptype == "max" else "avg")
        return self.module(mod, x, out_sp + (C,))

    def dense(self, x: Sym, features: int, act) -> Sym:
        fin = x.shape[-1]
        fused = act if act in (None, "relu", "tanh", "sigmoid", "softmax") else None
        mod = Dense(fin, features, act=fused)
        return self.module(mod, x, x.shape[:-1] + (features,), 2 * math.prod(x.shape[:-1]) * fin * features)

    # ----------------------------------------------------------------- IR elements
    def build_input(self, spec: InputSpec, x: Sym, neighbour: Sym | None, block_stride, block_features) -> Sym:
        kind = spec.kind
        if kind == "zeros":
            ref = neighbour if neighbour is not None else x
            return self.fn("zeros", None, (ref,), ref.shape, layer=False)
        if kind == "identity":
            return x
        stride = spec.stride
        if block_stride:
            stride = tuple(max(1, min(int(v), 2)) for v in block_stride)
        features = spec.features
        if block_features:
            features = max(MIN_FEATURES, min(int(x.shape[-1] * float(block_features)), MAX_FEATURES))
        if not features:
            features = MIN_FEATURES
        if kind == "dense":
            return self.dense(x, int(features), spec.activation)
        if kind == "convolution":
            if x.rank not in (3, 4, 5):
                return x
            if spec.type not in ("normal", "separable", "depthwise"):
                return x   # reference: unknown _type builds nothing (input.py:289-308)
            if spec.kernel is None:
                if not self.fill_defaults:
                    raise CompileError("convolution without kernel")
                spec = _with(spec, kernel=(3, 3))
            if x.rank == 3 and spec.type == "depthwise":
                return x
            kernel = spec.kernel
            if x.rank == 3:
                kernel = (int(kernel[0]),)
                stride = (int(_fit(stride or 1, 2)[0]),)
            return self.conv(x, int(features), kernel, stride, spec.padding or "same", spec.activation, spec.type)
        if kind == "pooling":
            if x.rank not in (4, 5):
                return x
            ptype = spec.type or "max"
            if ptype not in ("max", "average", "global"):
                return x
            if ptype != "global" and spec.kernel is None:
                if not self.fill_defaults:
                    raise CompileError("pooling without kernel")
                spec = _with(spec, kernel=(3, 3))
            return self.pool(x, spec.kernel, stride, ptype, spec.padding or "same")
        raise CompileError(f"unknown input kind {kind!r}")

    def build_op(self, spec: OpSpec, x: Sym) -> Sym:
        k = spec.kind
        if k == "void":
            return x
        if k == "flatten":
            return self.fn("flatten", None, (x,), (math.prod(x.shape),)) if x.rank > 2 else x
        if k == "dropout":
            if spec.value and spec.value > 0:
                return self.fn("dropout", float(spec.value), (x,), x.shape)
            return x
        if k == "padding":
            if x.rank != 4:
                return x
            ph, pw = (int(spec.fill_size[0]), int(spec.fill_size[1])) if spec.fill_size else (1, 1)
            h, w, c = x.shape
            return self.fn("pad", (ph, pw), (x,), (h + 2 * ph, w + 2 * pw, c))
        if k == "batchnorm":
            axis = spec.axis if self.compat else -1
            ax = axis if axis >= 0 else x.rank + axis
            if ax == 0 or ax >= x.rank:
                raise CompileError(f"batchnorm axis {axis} invalid for rank {x.rank}")
            ch = x.shape[ax - 1]
            mod = AxisBatchNorm(ch, axis=ax)
            return self.module(mod, x, x.shape)
        if k == "activation":
            return self.fn("act", spec.method or "relu", (x,), x.shape)
        raise CompileError(f"unknown operation {k!r}")

    def build_comb(self, comb, a: Sym, b: Sym) -> Sym:
        if a.rank == 4 and b.rank == 4 and a.shape[-1] != b.shape[-1]:
            if not a.shape[-1] < b.shape[-1]:
                a, b = b, a
            ratio = a.shape[1] / b.shape[1]
            dil, st = 1, ratio
            if st < 1:
                dil, st = 1 / st, 1
            st = int(st)
            mod = Conv(b.shape[-1], a.shape[-1], (1, 1, 1), (1, st, st), "valid", dilation=(1, int(dil), int(dil)),
                       act=None, bias=True)
            out_sp = tuple(_conv_out(i, 1, st, "valid") for i in b.shape[:-1])
            b = self.module(mod, b, out_sp + (a.shape[-1],), 2 * math.prod(out_sp) * a.shape[-1] * b.shape[-1])
        kind = comb.kind
        if kind == "sum":
            return self.fn("add", None, (a, b), a.shape) if a.shape == b.shape else b
        if kind == "concat":
            if a.shape != b.shape:
                return b
            axis = comb.axis if self.compat else -1
            ax = axis if axis >= 0 else a.rank + axis
            if ax == 0 or ax >= a.rank:
                raise CompileError("concat on the batch axis")
            shape = list(a.shape)
            shape[ax - 1] *= 2
            return self.fn("concat", ax, (a, b), tuple(shape))
        if kind == "product":
            if a.shape != b.shape:
                raise CompileError(f"Multiply of incompatible shapes {a.shape} vs {b.shape}")
            return self.fn("mul", None, (a, b), a.shape)
        raise CompileError(f"unknown combination {kind!r}")

    def build_cell(self, cell: CellSpec, stack: list, block_stride, block_features) -> list:
        cands = [e for e in stack if e.kind == "raw" or e.current == 0]
        if not cands:
            raise CompileError("cell has no available input")
        i1 = self.build_input(cell.input1, cands[0].sym, None, block_stride, block_features)
        o1 = self.build_op(cell.op1, i1)
        if cell.input2.kind == "zeros":
            comb = o1
        else:
            src2 = cands[1].sym if len(cands) > 1 else cands[0].sym
            i2 = self.build_input(cell.input2, src2, i1, block_stride, block_features)
            o2 = self.build_op(cell.op2, i2)
            comb = self.build_comb(cell.comb, o1, o2)
        outs = []
        if cell.output.kind == "cell":
            stack.insert(0, _Entry("cell", comb, int(cell.output.rel_cell_index)))
        elif cell.output.kind == "out":
            outs.insert(0, comb)
        return outs

    def build_block(self, block, stack: list) -> tuple[list, list]:
        block_input = stack[0]
        outputs = []
        for cell in block.cells:
            outputs += self.build_cell(cell, stack, block.stride, block.features)
            for e in stack:
                if e.kind == "cell" and e.current >= 0:
                    e.current -= 1
        return [_Entry("block", stack[0].sym, 0), block_input], outputs


def _with(spec: InputSpec, **kw) -> InputSpec:
    """Copy of ``spec`` with unpinned parameters filled (``fill_defaults``: the
    reference constructor defaults, ``model/input.py:194,246``)."""
    import dataclasses

    return dataclasses.replace(spec, **kw)


def _fit(v, nd: int) -> tuple:
    if isinstance(v, int):
        return (v,) * nd
    v = tuple(int(a) for a in v)
    if len(v) >= nd:
        return v[-nd:] if nd < len(v) else v
    return (v[0],) * (nd - len(v)) + v


def _pad3(v: tuple, fill: int) -> tuple:
    return (fill,) * (3 - len(v)) + tuple(v)


def _conv_out(i: int, k: int, s: int, pad: str) -> int:
    if pad == "same":
        return -(-i // s)
    return (i - k) // s + 1


def _pad_foldable(conv, extra) -> bool:
    """A ZeroPadding folds into ``conv`` only while every total pad stays within the kernel
    (lo, hi <= K - 1, stride 1, dilation 1): the stride-1 dgrad kernels run the transposed
    conv with leading pads K - 1 - lo, which must not go negative (a 1x1 conv after a
    fillSize-1 padding, or a 3x3 after padding 2, keeps the explicit pad op)."""
    strides = conv.stride if isinstance(conv.stride, (tuple, list)) else (conv.stride,) * 3
    dil = conv.dilation if isinstance(conv.dilation, (tuple, list)) else (conv.dilation,) * 3
    if any(int(v) != 1 for v in strides) or any(int(v) != 1 for v in dil):
        return False
    for k, e in zip(conv.kernel, extra):
        if conv.padding == "same":
            lo, hi = (k - 1) // 2, k - 1 - (k - 1) // 2
        elif conv.padding == "valid":
            lo, hi = 0, 0
        else:
            return False
        if lo + e > k - 1 or hi + e > k - 1:
            return False
    return True


class CandidateNet(nn.Module):
    """A compiled FeatureNet candidate: program over native-op modules."""

    def __init__(self, spec: ModelSpec, input_shape: tuple, n_classes: int, compat: bool = True,
                 max_params: int = MAX_PARAMS, fill_defaults: bool = False):
        super().__init__()
        b = _Builder(tuple(input_shape), compat, fill_defaults)
        stack = [_Entry("raw", b.x)]
        outputs: list = []
        for block in spec.blocks:
            stack, outs = b.build_block(block, stack)
            outputs += outs
        out = outputs[-1] if outputs else stack[0].sym
        if out.rank > 2:
            out = b.fn("flatten", None, (out,), (math.prod(out.shape),))
        head = Dense(out.shape[-1], n_classes, act=None)
        b.mods.append(head)
        b._emit(("head", len(b.mods) - 1, (out.node,)), (n_classes,),
                (sum(p.numel() for p in head.parameters()), 2 * out.shape[-1] * n_classes, 1))
        b.prune(len(b.prog) - 1)
        if b.params > max_params:
            raise ModelTooLarge(f"model has {b.params} parameters (> {max_params})")
        self.mods = b.mods
        self.prog = b.prog
        self.input_shape = tuple(input_shape)
        self.n_classes = n_classes
        self.nb_params = b.params
        self.nb_layers = b.layers
        self.flops_per_sample = b.flops
        self.spec_name = spec.name

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda and x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        # every conv weight pack of the candidate in one launch (ops/conv.py pack_scope; a no-op
        # on the CPU)
        with conv_ops.pack_scope(self):
            return self._run(x)

    def _run(self, x: torch.Tensor) -> torch.Tensor:
        vals: list = [None] * len(self.prog)
        for i, (kind, arg, ins) in enumerate(self.prog):
            if kind == "input":
                vals[i] = x
            elif kind == "module":
                vals[i] = self.mods[arg](vals[ins[0]])
            elif kind == "head":
                v = vals[ins[0]]
                vals[i] = self.mods[arg](v, out_fp32=True) if v.is_cuda else self.mods[arg](v).float()
            elif kind == "flatten":
                v = vals[ins[0]]
                vals[i] = v.reshape(v.shape[0], -1)
            elif kind == "gap":
                v = vals[ins[0]]
                vals[i] = v.reshape(v.shape[0], -1, v.shape[-1]).mean(1) if not v.is_cuda else \
                    ops.global_avg_pool(v.reshape(ops.to5d_shape(v.shape)))
            elif kind == "zeros":
                vals[i] = torch.zeros_like(vals[ins[0]])
            elif kind == "act":
                vals[i] = ops.activation(vals[ins[0]], arg)
            elif kind == "dropout":
                vals[i] = ops.dropout(vals[ins[0]], arg, self.training)
            elif kind == "alias":
                vals[i] = vals[ins[0]]
            elif kind == "pad":
                ph, pw = arg
                v = vals[ins[0]]
                n, h, w, c = v.shape
                vals[i] = ops.zero_pad(v.reshape(n, 1, h, w, c), (0, ph, pw)).reshape(n, h + 2 * ph, w + 2 * pw, c)
            elif kind == "add":
                vals[i] = ops.add(vals[ins[0]], vals[ins[1]])
            elif kind == "mul":
                vals[i] = ops.multiply(vals[ins[0]], vals[ins[1]])
            elif kind == "concat":
                vals[i] = ops.concat([vals[ins[0]], vals[ins[1]]], arg)
            else:  # pragma: no cover
                raise RuntimeError(f"bad instruction {kind}")
        return vals[-1]


def compile_model(spec: ModelSpec, input_shape: tuple, n_classes: int, compat: bool = True,
                  max_params: int = MAX_PARAMS, fill_defaults: bool = False) -> CandidateNet:
    """``compat`` keeps the reference's axis-1 BN/concat quirks; ``fill_defaults``
    gives unpinned kernels the reference constructor defaults instead of
    rejecting the candidate (the reference rejects it)."""
    try:
        return CandidateNet(spec, input_shape, n_classes, compat, max_params, fill_defaults)
    except CompileError:
        raise
    except Exception as e:  # any construction failure = invalid candidate
        raise CompileError(f"{type(e).__name__}: {e}") from e
