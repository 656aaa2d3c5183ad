"""Mutation and breeding operators over the architecture IR.

Reference parity (``model/mutation/*.py``): the operator lists, weights and
value tables are reproduced exactly; state that the reference kept in class
attributes (``MutableBase.mutation_stategy``, ``MAX_NB_CELLS``, ...) lives in
a :class:`MutationConfig` instance, and randomness comes from an explicit
``numpy.random.Generator`` so a search is reproducible from its seed.

Operator table (weights used by the CHOICE strategy; ALL applies every one):

=============  ==================================================  =====================
level          operators (weight)                                  reference
=============  ==================================================  =====================
model          add_block .3, mutate_block .5, remove_block .2      mutable_model.py:9
block          add_cell .3, mutate_cell .3, remove_cell .1,        mutable_block.py:14
               mutate_block_attrs .3
cell           mutate_input1 .4, mutate_input2 .3, mutate_output .3 mutable_cell.py:6
input          mutate_type .5, mutate_attributes .5                mutable_input.py:17
output         mutate_type .5, mutate_attributes .5                mutable_output.py:13
operation      mutate_type .5, mutate_attributes .5 (not reachable mutable_operation.py:13
               from cells, as in the reference)
combination    mutate_type 1 (unreachable in the reference)        mutable_combination.py:10
=============  ==================================================  =====================

Reference quirks kept on purpose (``compat`` semantics):
``remove_block`` is dead whenever the model has >= 1 block
(``mutable_model.py:40-41``); ``breed`` with the default ratio 1.0 clones
parent 1 (``:56-62``); a type mutation copies the old element's attribute
values onto the new element, so e.g. Identity -> Convolution yields a
convolution with ``type=None`` that builds nothing.
"""
from __future__ import annotations

import copy
import dataclasses
import enum
import math
from dataclasses import dataclass, field

import numpy as np

from ..ir.spec import BlockSpec, CellSpec, CombSpec, InputSpec, ModelSpec, OpSpec, OutSpec


class MutationStrategies(enum.Enum):
    CHOICE = 1
    ALL = 2


class SelectionStrategies(enum.Enum):
    ELITIST = 1
    HYBRID = 2
    PARETO = 3


# value tables (mutable_input.py:7-14, mutable_block.py:8-9, mutable_operation.py:7-9, mutable_output.py:7-8)
STRIDES_VALUES = ("1x1", "2x2")
FEATURES_MULTIPLIER_VALUES = (800, 400, 200, 100, 50, 25)
KERNEL_VALUES = ((1, 1), (3, 1), (1, 3), (3, 3), (5, 1), (1, 5), (5, 5), (7, 1), (1, 7), (7, 7))
POOL_TYPE_VALUES = ("max", "average", "global")
CONV_TYPE_VALUES = ("normal", "separable", "depthwise")
ACTIVATION_VALUES = ("relu", "sigmoid", None)
INPUT_ATTRIBUTES = {"kernel_values": ("kernel", KERNEL_VALUES), "pool_type_values": ("type", POOL_TYPE_VALUES),
                    "conv_type_values": ("type", CONV_TYPE_VALUES),
                    "activation_values": ("activation", ACTIVATION_VALUES)}
DROPOUT_VALUES = (0.7, 0.3, 0.5)
ACTIVATION_METHOD = ("relu", "tanh", "sigmoid")
CELL_INDEX_VALUES = (1, 2, 3)

MODEL_OPS = (("add_block", 0.3), ("mutate_block", 0.5), ("remove_block", 0.2))
BLOCK_OPS = (("add_cell", 0.3), ("mutate_cell", 0.3), ("remove_cell", 0.1), ("mutate_block_attrs", 0.3))
CELL_OPS = (("mutate_input1", 0.4), ("mutate_input2", 0.3), ("mutate_output", 0.3))
ELEMENT_OPS = (("mutate_type", 0.5), ("mutate_attributes", 0.5))


@dataclass
class MutationConfig:
    strategy: MutationStrategies = MutationStrategies.CHOICE
    selection: SelectionStrategies = SelectionStrategies.HYBRID
    max_nb_cells: int = 10
    max_nb_blocks: int = 20
    seed: int | None = None
    log: list = field(default_factory=list)


class Mutator:
    def __init__(self, config: MutationConfig | None = None, rng: np.random.Generator | None = None):
        self.cfg = config or MutationConfig()
        self.rng = rng or np.random.default_rng(self.cfg.seed)

    # ------------------------------------------------------------------ utils
    @property
    def choice_mode(self) -> bool:
        return self.cfg.strategy == MutationStrategies.CHOICE

    def _pick(self, ops):
        names = [o for o, _ in ops]
        w = np.array([p for _, p in ops], dtype=float)
        return names[self.rng.choice(len(names), p=w / w.sum())]

    def _apply(self, obj, ops, rate, handlers):
        if self.choice_mode:
            return [handlers[self._pick(ops)](obj, rate)]
        return [handlers[name](obj, rate) for name, _ in ops]

    def _note(self, *entry):
        self.cfg.log.append(entry)
        return entry

    # ------------------------------------------------------------------ model
    def mutate(self, model: ModelSpec, rate: float = 1.0):
        return self._apply(model, MODEL_OPS, rate, {
            "add_block": self.add_block, "mutate_block": self.mutate_block, "remove_block": self.remove_block})

    def add_block(self, model: ModelSpec, rate: float = 1.0):
        if len(model.blocks) >= self.cfg.max_nb_blocks:
            return self._note("add_block", None)
        if self.choice_mode or self.rng.random() < rate:
            idx = int(self.rng.integers(len(model.blocks))) if model.blocks else 0
            model.blocks.insert(idx, BlockSpec.base_block())
            return self._note("add_block", idx)
        return None

    def mutate_block(self, model: ModelSpec, rate: float = 1.0, block_index: int | None = None):
        if not model.blocks:
            return self._note("mutate_block", None)
        if block_index is None:
            if self.choice_mode:
                return self.mutate_block(model, rate, int(self.rng.integers(len(model.blocks))))
            return [self.mutate_block(model, rate, i) for i in range(len(model.blocks))]
        return self.mutate_block_ops(model.blocks[block_index], 1.0)   # reference calls block.mutate() (rate 1)

    def remove_block(self, model: ModelSpec, rate: float = 1.0, block_index: int | None = None):
        if len(model.blocks) >= 1:      # dead operator, as in the reference
            return self._note("remove_block", None)
        return None

    # ------------------------------------------------------------------ block
    def mutate_block_ops(self, block: BlockSpec, rate: float = 1.0):
        return self._apply(block, BLOCK_OPS, rate, {
            "add_cell": self.add_cell, "mutate_cell": self.mutate_cell, "remove_cell": self.remove_cell,
            "mutate_block_attrs": self.mutate_block_attrs})

    def add_cell(self, block: BlockSpec, rate: float = 1.0):
        if len(block.cells) >= self.cfg.max_nb_cells:
            return self._note("add_cell", None)
        if self.rng.random() < rate or self.choice_mode:
            idx = int(self.rng.integers(len(block.cells))) if block.cells else 0
            block.cells.insert(idx, CellSpec.base_cell())
            return self._note("add_cell", idx)
        return None

    def mutate_block_attrs(self, block: BlockSpec, rate: float = 1.0):
        out = []
        attrs = (("strides_values", STRIDES_VALUES, block.set_stride),
                 ("features_multiplier_values", FEATURES_MULTIPLIER_VALUES, block.set_features))
        if self.choice_mode:
            name, vals, setter = attrs[int(self.rng.integers(len(attrs)))]
            v = vals[int(self.rng.integers(len(vals)))]
            setter(v)
            out.append(self._note("mutate_block", name, v))
        else:
            for name, vals, setter in attrs:
                if self.rng.random() < rate:
                    v = vals[int(self.rng.integers(len(vals)))]
                    setter(v)
                    out.append(self._note("mutate_block", name, v))
        return out

    def mutate_cell(self, block: BlockSpec, rate: float = 1.0, cell_index: int | None = None):
        if not block.cells:
            return self._note("mutate_cell", None)
        if cell_index is not None:
            return self.mutate_cell_ops(block.cells[cell_index], rate)
        if self.choice_mode:
            return self.mutate_cell(block, rate, int(self.rng.integers(len(block.cells))))
        return [self.mutate_cell(block, rate, i) for i in range(len(block.cells))]

    def remove_cell(self, block: BlockSpec, rate: float = 1.0, cell_index: int | None = None):
        if not block.cells:
            return self._note("remove_cell", None)
        if cell_index is not None and 0 <= cell_index < len(block.cells):
            del block.cells[cell_index]
            return self._note("remove_cell", cell_index)
        if self.choice_mode:
            return self.remove_cell(block, rate, int(self.rng.integers(len(block.cells))))
        for i in range(len(block.cells)):
            if self.rng.random() < rate:
                return self.remove_cell(block, rate, i)
        return None

    # ------------------------------------------------------------------ cell
    def mutate_cell_ops(self, cell: CellSpec, rate: float = 1.0):
        return self._apply(cell, CELL_OPS, rate, {
            "mutate_input1": lambda c, r: self.mutate_input(c, "input1", r),
            "mutate_input2": lambda c, r: self.mutate_input(c, "input2", r),
            "mutate_output": self.mutate_output})

    # ------------------------------------------------------------------ inputs
    def mutate_input(self, cell: CellSpec, which: str, rate: float = 1.0):
        return self._apply(cell, ELEMENT_OPS, rate, {
            "mutate_type": lambda c, r: self.mutate_input_type(c, which, r),
            "mutate_attributes": lambda c, r: self.mutate_input_attributes(c, which, r)})

    def mutate_input_type(self, cell: CellSpec, which: str, rate: float = 1.0):
        if not (self.rng.random() < rate or self.choice_mode):
            return None
        kinds = ["identity", "convolution"]
        if which == "input2":
            kinds.append("zeros")              # only the second input may become Zeros
        kind = kinds[int(self.rng.integers(len(kinds)))]
        old: InputSpec = getattr(cell, which)
        new = _fresh_input(kind)
        # copy the attribute values (kernel/type/activation) of the previous input
        new.kernel, new.type, new.activation = old.kernel, old.type, old.activation
        setattr(cell, which, new)
        return self._note("mutate_input_type", which, kind)

    def mutate_input_attributes(self, cell: CellSpec, which: str, rate: float = 1.0):
        inp: InputSpec = getattr(cell, which)
        out = []
        keys = list(INPUT_ATTRIBUTES)
        if self.choice_mode:
            key = keys[int(self.rng.integers(len(keys)))]
            attr, vals = INPUT_ATTRIBUTES[key]
            v = vals[int(self.rng.integers(len(vals)))]
            setattr(inp, attr, v)
            out.append(self._note("mutate_input_attribute", key, v))
        else:
            for key in keys:
                if self.rng.random() < rate:
                    attr, vals = INPUT_ATTRIBUTES[key]
                    v = vals[int(self.rng.integers(len(vals)))]
                    setattr(inp, attr, v)
                    out.append(self._note("mutate_input_attribute", key, v))
        return out

    # ------------------------------------------------------------------ outputs
    def mutate_output(self, cell: CellSpec, rate: float = 1.0):
        return self._apply(cell, ELEMENT_OPS, rate, {
            "mutate_type": self.mutate_output_type, "mutate_attributes": self.mutate_output_attributes})

    def mutate_output_type(self, cell: CellSpec, rate: float = 1.0):
        if not (self.rng.random() < rate or self.choice_mode):
            return None
        kind = ("block", "cell")[int(self.rng.integers(2))]
        old = cell.output
        new = OutSpec(kind)
        # the reference copies _relativeCellIndex, which an OutBlock does not carry (None)
        new.rel_cell_index = old.rel_cell_index if old.kind == "cell" else None
        cell.output = new
        return self._note("mutate_output_type", kind)

    def mutate_output_attributes(self, cell: CellSpec, rate: float = 1.0):
        if self.choice_mode or self.rng.random() < rate:
            v = CELL_INDEX_VALUES[int(self.rng.integers(len(CELL_INDEX_VALUES)))]
            cell.output.rel_cell_index = v
            return [self._note("mutate_output_attribute", "cell_index_values", v)]
        return []

    # ------------------------------------------------------------------ operations / combinations
    def mutate_operation(self, cell: CellSpec, which: str = "op1", rate: float = 1.0):
        return self._apply(cell, ELEMENT_OPS, rate, {
            "mutate_type": lambda c, r: self.mutate_operation_type(c, which, r),
            "mutate_attributes": lambda c, r: self.mutate_operation_attributes(c, which, r)})

    def mutate_operation_type(self, cell: CellSpec, which: str = "op1", rate: float = 1.0):
        if not (self.rng.random() < rate or self.choice_mode):
            return None
        kind = ("activation", "batchnorm", "void", "dropout")[int(self.rng.integers(4))]
        old: OpSpec = getattr(cell, which)
        setattr(cell, which, OpSpec(kind, value=old.value, method=old.method))
        return self._note("mutate_operation_type", which, kind)

    def mutate_operation_attributes(self, cell: CellSpec, which: str = "op1", rate: float = 1.0):
        op: OpSpec = getattr(cell, which)
        table = (("dropout_values", "value", DROPOUT_VALUES), ("activation_method", "method", ACTIVATION_METHOD))
        out = []
        for i, (name, attr, vals) in enumerate(table):
            if self.choice_mode and i != int(self.rng.integers(len(table))):
                continue
            if self.choice_mode or self.rng.random() < rate:
                v = vals[int(self.rng.integers(len(vals)))]
                setattr(op, attr, v)
                out.append(self._note("mutate_operation_attribute", name, v))
            if self.choice_mode:
                break
        return out

    def mutate_combination(self, cell: CellSpec, rate: float = 1.0):
        if not (self.rng.random() < rate or self.choice_mode):
            return None
        kind = ("concat", "sum")[int(self.rng.integers(2))]
        cell.comb = CombSpec(kind, axis=cell.comb.axis)
        return self._note("mutate_combination_type", kind)

    # ------------------------------------------------------------------ evolution helpers
    def breed(self, parent1: ModelSpec, parent2: ModelSpec, ratio: float = 1.0) -> ModelSpec:
        b1 = copy.deepcopy(parent1.blocks)
        b2 = copy.deepcopy(parent2.blocks)
        child = ModelSpec()
        child.blocks = b1[: math.floor(len(b1) * ratio)] + b2[: math.ceil(len(b2) * (1 - ratio))]
        return child

    def generate_mutant(self, parent: ModelSpec, mutation_ratio: float, nb_max_mutations: int = 100) -> ModelSpec:
        """Reference ``FullEvolution.generate_mutant`` (``full_evolution.py:108-123``)."""
        if self.choice_mode:
            nb = int((self.rng.uniform(size=nb_max_mutations) < mutation_ratio).sum())
        else:
            nb = 1
        mutant = ModelSpec()
        mutant.blocks = copy.deepcopy(parent.blocks)
        for _ in range(nb):
            self.mutate(mutant, mutation_ratio)
        return mutant


def _fresh_input(kind: str) -> InputSpec:
    if kind == "convolution":
        return InputSpec.convolution()
    if kind == "zeros":
        return InputSpec.zeros()
    return InputSpec.identity()


def cell_signature(cell: CellSpec) -> dict:
    return dataclasses.asdict(cell)
