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


def test_lenet5_param_count_pinned():
    # Regression pin of our compile semantics for the reference LeNet-5 template on
    # MNIST (parity with the TF build is unpinned: TF is not importable here).
    net = compile_model(parse_feature_model("lenet5", name="lenet5"), (28, 28, 1), 10)
    assert net.nb_params == 212902


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
