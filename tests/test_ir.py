"""IR: product -> spec parsing, templates, compile (shape/param inference), spec JSON."""
import os

import pytest
import torch

from featurenet_amd.fm.products import ProductSet
from featurenet_amd.ir.compile import CompileError, ModelTooLarge, compile_model
from featurenet_amd.ir.parse import parse_feature_model
from featurenet_amd.ir.spec import ModelSpec

REF = "/root/reference"
need_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="reference fixtures not present")


def _check_net(net, shape, ncls, batch=3):
    x = torch.rand((batch,) + tuple(shape))
    y = net(x)
    assert y.shape == (batch, ncls)
    assert torch.isfinite(y).all()
    # Keras count_params semantics: BN moving statistics count as (non-trainable) params
    n = sum(p.numel() for p in net.parameters())
    n += sum(b.numel() for name, b in net.named_buffers() if name.endswith(("running_mean", "running_var")))
    assert n == net.nb_params
    y.float().sum().backward()
    # dead branches are pruned; only layers feeding a ``zeros`` input (shape-only
    # dependency, still part of the Keras graph) may go without a gradient
    feeds_zeros = {j for kind, _, ins in net.prog if kind == "zeros" for j in ins}
    zero_mods = {net.prog[j][1] for j in feeds_zeros if net.prog[j][0] == "module"}
    for i, m in enumerate(net.mods):
        if i not in zero_mods:
            assert all(p.grad is not None for p in m.parameters() if p.requires_grad), f"module {i} has no grad"
    return y


@pytest.mark.parametrize("name,shape,ncls", [("lenet5", (28, 28, 1), 10), ("lenet5", (32, 32, 3), 10),
                                             ("keras", (32, 32, 3), 10), ("keras", (28, 28, 1), 10)])
def test_templates_compile(name, shape, ncls):
    spec = parse_feature_model(name, name=name)
    net = compile_model(spec, shape, ncls)
    _check_net(net, shape, ncls)
    assert net.nb_layers > 3
    assert net.flops_per_sample > 0


def _keras_lenet5_params(h: int, w: int, c: int, ncls: int) -> int:
    """Keras parameter count of the reference ``lenet5_blocks()`` template (model/leNet.py:7-40),
    derived by hand from the reference build semantics -- TF/Keras is not importable here, so
    this arithmetic IS the parity oracle:

    * block1 (stride 1x1, features 600 -> multiplier 6.0, model/block.py:31-35):
      cell11 ConvolutionInput 5x5 'same' tanh with no own feature count, so the block's
      multiplier applies: features = in_channels * 6 clamped to [6, 2048] (model/input.py:30-40)
      -> Conv2D(6c, 5x5): 25*c*6c + 6c.  cell12 AveragePooling 2x2 -- its 'valid' padding is
      not an accepted value and becomes 'same' (model/input.py:201-211), stride 1x1 from the
      block -> h x w x 6c, no parameters.  cell12 reads cell11's output: the default OutCell
      (index 1, model/output.py:81-95) is pushed on the stack front and counted down to 0
      after cell11 (model/block.py:58-60, model/cell.py:49,76-82).
    * block2 (stride 1x1, no multiplier): Conv2D(12, 5x5 'same') on 6c channels: 25*6c*12 + 12.
    * block22 (stride 2x2): AveragePooling 2x2 'same' stride 2 -> ceil(h/2) x ceil(w/2).
    * block3: ConvolutionInput 5x5 'valid' -> 'same' (model/input.py:264-275): Conv2D(120):
      25*12*120 + 120.
    * block4: DenseInput(84, tanh) on the 4-D tensor (last axis, model/input.py:190): 120*84 + 84.
    * head: Flatten + Dense(ncls) (model/keras_model.py:118-124): ceil(h/2)*ceil(w/2)*84*ncls + ncls.
    """
    f1 = 6 * c
    conv1 = 25 * c * f1 + f1
    conv2 = 25 * f1 * 12 + 12
    conv3 = 25 * 12 * 120 + 120
    dense = 120 * 84 + 84
    head = -(-h // 2) * -(-w // 2) * 84 * ncls + ncls
    return conv1 + conv2 + conv3 + dense + head


@pytest.mark.parametrize("shape,ncls", [((28, 28, 1), 10), ((32, 32, 3), 10), ((32, 32, 3), 100)])
def test_lenet5_param_count_matches_hand_derived_keras(shape, ncls):
    net = compile_model(parse_feature_model("lenet5", name="lenet5"), shape, ncls)
    expected = _keras_lenet5_params(*shape, ncls)
    assert net.nb_params == expected
    if shape == (28, 28, 1):
        # 156 + 1812 + 36120 + 10164 + 164650
        assert expected == 212902


def test_featurenet3d_template_compiles_3d():
    spec = parse_feature_model("featurenet3d", name="fn3d")
    net = compile_model(spec, (32, 32, 32, 1), 4, compat=False, fill_defaults=True)
    _check_net(net, (32, 32, 32, 1), 4, batch=2)


def test_spec_json_roundtrip():
    spec = parse_feature_model("keras", name="k")
    spec.accuracy = 0.5
    s2 = ModelSpec.from_json(spec.to_json())
    assert s2.to_dict() == spec.to_dict()
    a = compile_model(spec, (32, 32, 3), 10)
    b = compile_model(s2, (32, 32, 3), 10)
    assert a.nb_params == b.nb_params


def test_model_too_large():
    spec = parse_feature_model("keras", name="k")
    with pytest.raises(ModelTooLarge):
        compile_model(spec, (32, 32, 3), 10, max_params=1000)


@need_ref
def test_product0_has_ten_blocks():
    ps = ProductSet(f"{REF}/datasets/10Products.pdt")
    tree, feats = ps.format_product(0)
    spec = parse_feature_model(tree, name="p0", product_features=sorted(feats, key=lambda k: abs(int(k))))
    assert len(spec.blocks) == 10
    assert len(spec.features) == ps.nbFeatures
    assert spec.nb_cells() > 10


@need_ref
def test_pdt_products_compile_with_defaults():
    """All 10 real PLEDGE products build once unpinned kernels get constructor defaults.

    Without ``fill_defaults`` these products carry poolings without a kernel size,
    which the reference rejects too (its candidate is dropped), so they raise
    :class:`CompileError` here.
    """
    ps = ProductSet(f"{REF}/datasets/10Products.pdt")
    built, rejected = 0, 0
    for i, (tree, _) in enumerate(ps.format_products()):
        spec = parse_feature_model(tree, name=f"p{i}")
        try:
            compile_model(spec, (32, 32, 3), 10)
        except CompileError:
            rejected += 1
        net = compile_model(spec, (32, 32, 3), 10, fill_defaults=True)
        _check_net(net, (32, 32, 3), 10, batch=2)
        built += 1
    assert built == 10
    assert rejected >= 1
