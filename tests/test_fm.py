"""Feature-model layer: SPLOT parsing, extender goldens, .pdt IO, CNF, sampler.

Goldens are the reference's own fixtures (read as text only):
``main_1block_nas.xml`` -> ``nas_1_1_10.xml`` (byte-exact),
``main_1block_nas.xml`` + block features -> ``nas_5_5_10.xml`` (tree + constraints),
``datasets/10Products.pdt`` (real PLEDGE output).
"""
import os
import random
import xml.etree.ElementTree as ET

import pytest

from featurenet_amd.fm import extend, splot
from featurenet_amd.fm.products import ProductSet

REF = "/root/reference"
need_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="reference fixtures not present")


@need_ref
def test_extender_1x1_byte_exact(tmp_path):
    out = tmp_path / "nas_1_1_10.xml"
    extend.generate_featuretree(f"{REF}/main_1block_nas.xml", out, 1, 1)
    assert out.read_bytes() == open(f"{REF}/nas_1_1_10.xml", "rb").read()


@need_ref
def test_extender_5x5_block_features(tmp_path):
    out = tmp_path / "nas_5_5.xml"
    extend.generate_featuretree(f"{REF}/main_1block_nas.xml", out, 5, 5, block_features=True)
    got, want = list(ET.parse(out).getroot()), list(ET.parse(f"{REF}/nas_5_5_10.xml").getroot())
    assert got[0].text.strip() == want[0].text.strip()
    assert got[1].text.strip() == want[1].text.strip()


@need_ref
def test_splot_parse_and_cnf():
    fm = splot.load(f"{REF}/nas_1_1_10.xml")
    names = fm.names()
    assert names[0] == fm.root.name
    assert len(names) == len(set(names))
    nvars, clauses = fm.to_cnf()
    assert nvars == len(names)
    assert all(all(1 <= abs(l) <= nvars for l in c) for c in clauses)
    # the root is forced
    assert [1] in clauses
    # xml round trip keeps the tree
    fm2 = splot.loads(splot.to_xml(fm))
    assert fm2.names() == names


def test_splot_group_semantics():
    xml = """<?xml version="1.0"?>
<featureModel><feature_tree>
:r R(R)
\t:m A(A)
\t\t:g [1,1]
\t\t\t: A1(A1)
\t\t\t: A2(A2)
\t:o B(B)
</feature_tree><constraints>
C1:~B or A2
</constraints></featureModel>"""
    fm = splot.loads(xml)
    assert fm.is_valid({"R", "A", "A1"})
    assert not fm.is_valid({"R", "A", "A1", "A2"})        # xor group
    assert not fm.is_valid({"R", "A"})                    # group needs one member
    assert not fm.is_valid({"R", "A", "A1", "B"})         # cross-tree constraint
    assert fm.is_valid({"R", "A", "A2", "B"})


@need_ref
def test_pdt_roundtrip(tmp_path):
    ps = ProductSet(f"{REF}/datasets/10Products.pdt")
    assert ps.nbProducts == 10
    assert ps.nbFeatures > 6000
    labels = [ps.features[str(i + 1)] for i in range(ps.nbFeatures)]
    ProductSet.write(tmp_path / "rt.pdt", labels, [[int(t) for t in p] for p in ps.products])
    ps2 = ProductSet(tmp_path / "rt.pdt")
    assert ps2.features == ps.features
    assert [[int(t) for t in p] for p in ps2.products] == [[int(t) for t in p] for p in ps.products]
    psb = ProductSet(f"{REF}/datasets/10Products.pdt", binary_products=True)
    assert all(len(p) == ps.nbFeatures for p in psb.products)
    assert psb.products[0] == ps.binary_vector(ps.products[0])


@need_ref
def test_product_tree_blocks():
    ps = ProductSet(f"{REF}/datasets/10Products.pdt")
    blocks, feats = ps.format_product(0)
    assert len(blocks) == 10          # 10 blocks for product 0
    assert all(b["label"].startswith("Block") for b in blocks)
    light = ps.light_product(0)
    assert len(light) == 10


def _rt():
    from featurenet_amd import _native

    if not _native.runtime_available():
        pytest.skip("native runtime not built")
    return _native.runtime()


def test_native_sampler_products_are_valid():
    rt = _rt()
    xml = open(f"{REF}/nas_1_1_10.xml").read() if os.path.isdir(REF) else None
    if xml is None:
        pytest.skip("no fixture")
    fm = splot.loads(xml)
    nvars, clauses = fm.to_cnf()
    names = fm.names()
    res = rt.sample_diverse(nvars, clauses, 12, 200.0, 3, 0, True)
    prods = res["products"]
    assert len(prods) == 12
    for p in prods:
        sel = {names[abs(v) - 1] for v in p if v > 0}
        assert fm.is_valid(sel)
        assert rt.check(nvars, clauses, p)
    assert res["fitness"] >= res["initial_fitness"]


def test_sampler_random_cnf_agrees_with_python_check():
    rt = _rt()
    rng = random.Random(5)
    nv = 30
    clauses = [[rng.choice([-1, 1]) * rng.randint(1, nv) for _ in range(3)] for _ in range(60)]
    prods = rt.random_products(nv, clauses, 8, 1)
    for p in prods:
        val = {abs(v): v > 0 for v in p}
        assert all(any(val[abs(l)] == (l > 0) for l in c) for c in clauses)


@need_ref
def test_run_pledge_writes_loadable_pdt(tmp_path):
    _rt()
    from featurenet_amd.fm.sampler import run_pledge

    out = tmp_path / "p.pdt"
    assert run_pledge(f"{REF}/nas_1_1_10.xml", 5, out, duration=0.2) == 0
    ps = ProductSet(out)
    assert ps.nbProducts == 5
    fm = splot.load(f"{REF}/nas_1_1_10.xml")
    for p in ps.products:
        assert fm.is_valid(set(ps.enabled_labels(p)))
