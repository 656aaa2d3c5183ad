"""Architecture IR: the block / cell / input / operation / combination / output
hierarchy of a FeatureNet candidate as plain, JSON-serialisable data.

Reference parity (``model/*.py``): ``Block`` (``block.py:8``), ``Cell``
(``cell.py:8``), the ``Input`` family (``input.py:11-308``), ``Operation``
(``operation.py:10-165``), ``Combination`` (``operation.py:168-248``) and
``Output`` (``output.py:7-95``).  The reference mixes these with Keras graph
construction and class-level mutable state; here the IR is inert data and
:mod:`featurenet_amd.ir.compile` lowers it to a module of native ops.

Attribute names follow the reference's private attributes (``_kernel``,
``_type``, ...) without the underscore, because the mutation value tables
address them by those names (``model/mutation/mutable_input.py:7-14``).
"""
from __future__ import annotations

import copy
import itertools
import json
from dataclasses import asdict, dataclass, field
from typing import Any

_ids = itertools.count(1)


def _new_id() -> str:
    return f"n{next(_ids):06d}"


# ---------------------------------------------------------------------------
# inputs
# ---------------------------------------------------------------------------
INPUT_KINDS = ("identity", "zeros", "convolution", "pooling", "dense")


@dataclass
class InputSpec:
    kind: str = "identity"
    kernel: Any = None            # (kh, kw) tuple or None
    stride: Any = None            # (sh, sw) tuple, int or None (-> 1)
    features: Any = None          # absolute feature count or None
    padding: str | None = "same"
    activation: str | None = "relu"
    type: str | None = None       # conv: normal|separable|depthwise ; pool: max|average|global
    custom: dict = field(default_factory=dict)   # unpinned parameters (get_custom_parameters)
    label: str = ""

    @staticmethod
    def identity() -> "InputSpec":
        return InputSpec("identity", activation=None)

    @staticmethod
    def zeros() -> "InputSpec":
        return InputSpec("zeros", activation=None)

    @staticmethod
    def convolution(kernel=(3, 3), stride=(1, 1), features=8, padding="same", activation="relu",
                    type="normal") -> "InputSpec":
        return InputSpec("convolution", kernel=tuple(kernel) if kernel else None,
                         stride=tuple(stride) if stride else None, features=features, padding=padding,
                         activation=activation, type=type)

    @staticmethod
    def pooling(kernel=(3, 3), stride=(1, 1), type="max", padding="same") -> "InputSpec":
        return InputSpec("pooling", kernel=tuple(kernel) if kernel else None, stride=tuple(stride) if stride else None,
                         padding=padding, activation=None, type=type)

    @staticmethod
    def dense(features=128, activation="relu") -> "InputSpec":
        return InputSpec("dense", features=features, activation=activation)


# ---------------------------------------------------------------------------
# operations, combinations, outputs
# ---------------------------------------------------------------------------
OP_KINDS = ("void", "flatten", "dropout", "padding", "batchnorm", "activation")


@dataclass
class OpSpec:
    kind: str = "void"
    value: float = 0.0            # dropout rate
    fill_size: Any = (1, 1)       # zero padding
    axis: int = 1                 # BN axis (reference forces 1)
    method: str | None = "relu"   # activation
    label: str = ""


COMB_KINDS = ("sum", "concat", "product")


@dataclass
class CombSpec:
    kind: str = "sum"
    axis: int = 1                 # concat axis (reference forces 1)
    label: str = ""


OUT_KINDS = ("cell", "block", "out")


@dataclass
class OutSpec:
    kind: str = "cell"
    rel_cell_index: int = 1       # stored +1 like the reference (_relativeCellIndex)
    rel_block_index: int = 0
    label: str = ""


# ---------------------------------------------------------------------------
# cells, blocks, models
# ---------------------------------------------------------------------------
@dataclass
class CellSpec:
    input1: InputSpec = field(default_factory=InputSpec.identity)
    input2: InputSpec = field(default_factory=InputSpec.zeros)
    op1: OpSpec = field(default_factory=OpSpec)
    op2: OpSpec = field(default_factory=OpSpec)
    comb: CombSpec = field(default_factory=CombSpec)
    output: OutSpec = field(default_factory=OutSpec)
    name: str = field(default_factory=_new_id)

    @staticmethod
    def base_cell() -> "CellSpec":
        """Reference ``Cell.base_cell`` (``model/cell.py:98-102``): 3x3/s1 conv, 8 filters, same, relu."""
        return CellSpec(input1=InputSpec.convolution((3, 3), (1, 1), 8, "same", "relu"))


@dataclass
class BlockSpec:
    cells: list = field(default_factory=list)
    stride: Any = None            # ("2","2") style list like the reference, or None
    features: float | None = None  # relative features multiplier (800 -> 8.0)
    name: str = field(default_factory=_new_id)

    def set_stride(self, s: str) -> None:
        self.stride = s.split("x")

    def set_features(self, f) -> None:
        self.features = int(f) / 100

    @staticmethod
    def base_block() -> "BlockSpec":
        return BlockSpec(cells=[CellSpec.base_cell()])


@dataclass
class ModelSpec:
    blocks: list = field(default_factory=list)
    name: str = field(default_factory=lambda: _new_id())
    features: list = field(default_factory=list)        # 0/1 product bit vector
    features_label: list = field(default_factory=list)
    # results (KerasFeatureModel class attributes in the reference)
    accuracy: float = 0.0
    nb_params: int = 0
    nb_flops: int = 0
    nb_layers: int = 0
    robustness_score: float = 0.0
    clever_score: float = 0.0
    fgsm_score: Any = 0.0
    pgd_score: Any = 0.0
    cw_score: Any = 0.0
    metrics: list = field(default_factory=list)
    history: dict = field(default_factory=dict)
    status: str = "new"                                  # new | trained | invalid | failed
    error: str = ""

    # ------------------------------------------------------------ helpers
    def clone(self) -> "ModelSpec":
        return copy.deepcopy(self)

    def nb_cells(self) -> int:
        return sum(len(b.cells) for b in self.blocks)

    def to_dict(self) -> dict:
        return _todict(self)

    def to_json(self) -> str:
        return json.dumps(self.to_dict())

    @staticmethod
    def from_dict(d: dict) -> "ModelSpec":
        blocks = []
        for b in d.get("blocks", []):
            cells = []
            for c in b.get("cells", []):
                cells.append(CellSpec(
                    input1=_mk(InputSpec, c["input1"]), input2=_mk(InputSpec, c["input2"]),
                    op1=_mk(OpSpec, c["op1"]), op2=_mk(OpSpec, c["op2"]), comb=_mk(CombSpec, c["comb"]),
                    output=_mk(OutSpec, c["output"]), name=c.get("name", _new_id())))
            blocks.append(BlockSpec(cells=cells, stride=b.get("stride"), features=b.get("features"),
                                    name=b.get("name", _new_id())))
        kw = {k: v for k, v in d.items() if k != "blocks" and k in ModelSpec.__dataclass_fields__}
        return ModelSpec(blocks=blocks, **kw)

    @staticmethod
    def from_json(s: str) -> "ModelSpec":
        return ModelSpec.from_dict(json.loads(s))


def _todict(o):
    if hasattr(o, "__dataclass_fields__"):
        return {k: _todict(getattr(o, k)) for k in o.__dataclass_fields__}
    if isinstance(o, (list, tuple)):
        return [_todict(v) for v in o]
    if isinstance(o, dict):
        return {k: _todict(v) for k, v in o.items()}
    return o


def _mk(cls, d: dict):
    kw = {k: v for k, v in d.items() if k in cls.__dataclass_fields__}
    for k in ("kernel", "stride", "fill_size"):
        if k in kw and isinstance(kw[k], list):
            kw[k] = tuple(kw[k])
    return cls(**kw)
