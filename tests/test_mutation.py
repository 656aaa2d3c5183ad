"""Mutation / breeding operators and survivor selection (seeded, deterministic)."""
from collections import Counter

import numpy as np
import pytest

from featurenet_amd.ir.compile import CompileError, compile_model
from featurenet_amd.ir.parse import parse_feature_model
from featurenet_amd.ir.spec import BlockSpec, CellSpec, InputSpec, ModelSpec
from featurenet_amd.search import mutation as M
from featurenet_amd.search.selection import get_fronts, select


def _lenet():
    return parse_feature_model("lenet5", name="lenet5")


def _strip(d):
    """Spec dict without the auto-generated element names."""
    if isinstance(d, dict):
        return {k: _strip(v) for k, v in d.items() if k != "name"}
    if isinstance(d, list):
        return [_strip(v) for v in d]
    return d


def _mut(seed=0, strategy=M.MutationStrategies.CHOICE, **kw):
    return M.Mutator(M.MutationConfig(strategy=strategy, seed=seed, **kw))


def test_operator_weights_match_reference_tables():
    assert dict(M.MODEL_OPS) == {"add_block": 0.3, "mutate_block": 0.5, "remove_block": 0.2}
    assert dict(M.BLOCK_OPS) == {"add_cell": 0.3, "mutate_cell": 0.3, "remove_cell": 0.1, "mutate_block_attrs": 0.3}
    assert dict(M.CELL_OPS) == {"mutate_input1": 0.4, "mutate_input2": 0.3, "mutate_output": 0.3}
    assert M.FEATURES_MULTIPLIER_VALUES == (800, 400, 200, 100, 50, 25)
    assert len(M.KERNEL_VALUES) == 10


def test_pick_follows_weights():
    m = _mut(1)
    c = Counter(m._pick(M.MODEL_OPS) for _ in range(20000))
    assert abs(c["add_block"] / 20000 - 0.3) < 0.02
    assert abs(c["mutate_block"] / 20000 - 0.5) < 0.02


def test_add_block_respects_cap():
    s = _lenet()
    n0 = len(s.blocks)
    m = _mut(0, max_nb_blocks=n0 + 1)
    assert m.add_block(s)[1] is not None
    assert len(s.blocks) == n0 + 1
    assert m.add_block(s) == ("add_block", None)       # at the cap
    assert len(s.blocks) == n0 + 1


def test_remove_block_is_dead_like_reference():
    s = _lenet()
    n = len(s.blocks)
    _mut(0).remove_block(s)
    assert len(s.blocks) == n


def test_cell_ops_and_caps():
    m = _mut(3, max_nb_cells=2)
    b = BlockSpec(cells=[CellSpec.base_cell()])
    m.add_cell(b)
    assert len(b.cells) == 2
    assert m.add_cell(b) == ("add_cell", None)
    m.remove_cell(b, cell_index=0)
    assert len(b.cells) == 1


def test_block_attribute_domains():
    m = _mut(4)
    b = BlockSpec.base_block()
    for _ in range(50):
        m.mutate_block_attrs(b)
    names = {e[1] for e in m.cfg.log if e[0] == "mutate_block"}
    assert names <= {"strides_values", "features_multiplier_values"}
    vals = [e[2] for e in m.cfg.log if e[0] == "mutate_block"]
    assert all(v in M.STRIDES_VALUES + M.FEATURES_MULTIPLIER_VALUES for v in vals)


def test_input_type_domain():
    m = _mut(5)
    seen1, seen2 = set(), set()
    for _ in range(60):
        c = CellSpec.base_cell()
        m.mutate_input_type(c, "input1")
        m.mutate_input_type(c, "input2")
        seen1.add(c.input1.kind)
        seen2.add(c.input2.kind)
    assert seen1 == {"identity", "convolution"}
    assert seen2 == {"identity", "convolution", "zeros"}


def test_input_attribute_domain():
    m = _mut(6)
    c = CellSpec(input1=InputSpec.convolution())
    for _ in range(100):
        m.mutate_input_attributes(c, "input1")
        assert c.input1.kernel is None or tuple(c.input1.kernel) in M.KERNEL_VALUES
        assert c.input1.activation in M.ACTIVATION_VALUES
        assert c.input1.type in M.POOL_TYPE_VALUES + M.CONV_TYPE_VALUES


def test_output_ops():
    m = _mut(7)
    c = CellSpec.base_cell()
    for _ in range(30):
        m.mutate_output(c)
        assert c.output.kind in ("block", "cell")
        if c.output.rel_cell_index is not None:
            assert c.output.rel_cell_index in M.CELL_INDEX_VALUES


def test_operation_and_combination_ops():
    m = _mut(8)
    c = CellSpec.base_cell()
    for _ in range(20):
        m.mutate_operation(c, "op1")
        m.mutate_combination(c)
        assert c.op1.kind in ("activation", "batchnorm", "void", "dropout")
        assert c.comb.kind in ("concat", "sum")


def test_breed_ratio_one_clones_parent1():
    m = _mut(0)
    a, b = _lenet(), parse_feature_model("keras", name="keras")
    child = m.breed(a, b)
    assert [x.to_dict() if hasattr(x, "to_dict") else x for x in child.blocks] == \
           [x.to_dict() if hasattr(x, "to_dict") else x for x in a.blocks]
    half = m.breed(a, b, ratio=0.5)
    assert len(half.blocks) == len(a.blocks) // 2 + (len(b.blocks) + 1) // 2


def test_generate_mutant_deterministic_and_mostly_buildable():
    a = _lenet()
    m1, m2 = _mut(11), _mut(11)
    built = 0
    for _ in range(20):
        x = m1.generate_mutant(a, 0.1)
        y = m2.generate_mutant(a, 0.1)
        assert _strip(x.to_dict()) == _strip(y.to_dict())
        try:
            compile_model(x, (28, 28, 1), 10)
            built += 1
        except CompileError:
            pass
    assert built >= 10          # "mutants still build" (reference tests_mutant.py)
    assert _strip(a.to_dict()) == _strip(_lenet().to_dict())     # parent untouched


def test_all_strategy_applies_every_operator():
    m = _mut(0, strategy=M.MutationStrategies.ALL)
    s = _lenet()
    res = m.mutate(s, 1.0)
    assert len(res) == 3


# ---------------------------------------------------------------------- selection
class _P:
    def __init__(self, acc, rob=0.0):
        self.accuracy, self.robustness_score = acc, rob


def test_fronts():
    acc = [0.9, 0.8, 0.7, 0.95]
    rob = [0.1, 0.5, 0.4, 0.05]
    assert get_fronts(acc, rob) == [0, 1, 3]


@pytest.mark.parametrize("strategy", list(M.SelectionStrategies))
def test_select_sizes(strategy):
    pop = sorted([_P(a, r) for a, r in zip(np.linspace(0.2, 0.9, 10), np.linspace(0.5, 0.1, 10))],
                 key=lambda p: -p.accuracy)
    out = select(pop, 4, strategy, np.random.default_rng(0))
    assert len(out) == 4 if strategy != M.SelectionStrategies.PARETO else 1 <= len(out) <= 4
    if strategy == M.SelectionStrategies.ELITIST:
        assert [p.accuracy for p in out] == [p.accuracy for p in pop[:4]]
