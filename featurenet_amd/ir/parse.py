"""Product tree (``{"label","id","children"}`` dicts, see
:mod:`featurenet_amd.fm.products`) -> :class:`~featurenet_amd.ir.spec.ModelSpec`.

Reference parity: ``KerasFeatureModel.parse_feature_model``
(``model/keras_model.py:176-205``), ``Block.parse_feature_model``
(``model/block.py:87-113``), ``Cell.parse_feature_model`` (``model/cell.py:105-138``),
``Input/Operation/Combination/Output.parse_feature_model``.

Label conventions: an element's *type* is its label suffix after the last
``_`` (lower-cased for inputs/operations); block attribute children are
``..._stride_<SxS>`` / ``..._features_<int>``; a cell lives under
``BlockK_ElementI`` -> ``BlockK_ElementI_Cell``.  Values the product leaves
unpinned become ``custom`` entries (the reference's "customizable
parameters", ``model/node.py:29-38``).
"""
from __future__ import annotations

import copy

from .spec import BlockSpec, CellSpec, CombSpec, InputSpec, ModelSpec, OpSpec, OutSpec

ACT_VALUES = ("tanh", "relu", "sigmoid", "softmax", "none")


def get_type(node: dict, keep_index: bool = True) -> str:
    lab = node.get("label", "")
    t = lab[lab.rfind("_") + 1:]
    if not keep_index:
        t = "".join(ch for ch in t if not ch.isdigit())
    return t.lower()


def _first_child_type(node: dict) -> str | None:
    ch = node.get("children") or []
    return get_type(ch[0]) if ch else None


def _pair(v: str | None):
    if not v:
        return None
    parts = v.split("x")
    return tuple(parts) if len(parts) == 2 else None


# ---------------------------------------------------------------------------
def parse_input(node: dict) -> InputSpec | None:
    children = node.get("children") or []
    if not children:
        return None
    inp = children[0]
    kind = get_type(inp)
    lab = inp.get("label", "")
    if kind == "zeros":
        return InputSpec("zeros", activation=None, label=lab)
    if kind == "identity":
        return InputSpec("identity", activation=None, label=lab)
    attrs: dict[str, str | None] = {}
    for ch in inp.get("children") or []:
        attrs[get_type(ch)] = _first_child_type(ch)
    if kind == "dense":
        spec = InputSpec("dense", label=lab)
        feats, act = attrs.get("features"), attrs.get("activation")
        if not feats:
            spec.custom["features"] = "__int__"
        else:
            spec.features = int(feats)
        if not act or act not in ACT_VALUES:
            spec.custom["activation"] = "|".join(ACT_VALUES)
            spec.activation = "relu"
        else:
            spec.activation = None if act == "none" else act
        return spec
    if kind == "pooling":
        spec = InputSpec("pooling", activation=None, label=lab)
        t = attrs.get("type")
        if not t or t not in ("max", "average", "global"):
            spec.custom["type"] = "max|average|global"
            spec.type = "max"
        else:
            spec.type = t
        if spec.type != "global":
            k = _pair(attrs.get("kernel"))
            if not k:
                spec.custom["kernel"] = "(__int__,__int__)"
            else:
                spec.kernel = (min(int(k[0]), 3), min(int(k[1]), 3))
            s = _pair(attrs.get("stride"))
            if not s:
                spec.custom["stride"] = "(__int__,__int__)"
            else:
                spec.stride = (int(s[0]), int(s[1]))
            p = attrs.get("padding")
            if p != "same":
                spec.custom["padding"] = "same"
            spec.padding = "same"
        return spec
    if kind == "convolution":
        spec = InputSpec("convolution", label=lab)
        t = attrs.get("type")
        if not t or t not in ("normal", "separable", "depthwise"):
            spec.custom["type"] = "normal|separable|depthwise"
            spec.type = "normal"
        else:
            spec.type = t
        k = _pair(attrs.get("kernel"))
        if not k:
            spec.custom["kernel"] = "(__int__,__int__)"
        else:
            spec.kernel = (min(int(k[0]), 5), min(int(k[1]), 5))
        s = _pair(attrs.get("stride"))
        if not s:
            spec.custom["stride"] = "(__int__,__int__)"
        else:
            spec.stride = (int(s[0]), int(s[1]))
        f = attrs.get("features")
        if not f:
            spec.custom["features"] = "__int__"
        else:
            spec.features = int(f)
        act = attrs.get("activation", "relu") or "relu"
        if act not in ACT_VALUES:
            spec.custom["activation"] = "|".join(ACT_VALUES)
        else:
            spec.activation = None if act == "none" else act
        p = attrs.get("padding")
        if p != "same":
            spec.custom["padding"] = "same"
        spec.padding = "same"
        return spec
    return None


def parse_operation(node: dict) -> OpSpec | None:
    children = node.get("children") or []
    if not children:
        return None
    op = children[0]
    kind = get_type(op)
    lab = op.get("label", "")
    attrs = {get_type(ch): _first_child_type(ch) for ch in op.get("children") or []}
    if kind == "void":
        return OpSpec("void", label=lab)
    if kind == "flatten":
        return OpSpec("flatten", label=lab)
    if kind == "dropout":
        v = attrs.get("value")
        return OpSpec("dropout", value=(int(v) / 100 if v else 0.0), label=lab)
    if kind == "padding":
        fs = _pair(attrs.get("fillsize"))
        return OpSpec("padding", fill_size=(int(fs[0]), int(fs[1])) if fs else (1, 1), label=lab)
    if kind == "batchnormalization":
        return OpSpec("batchnorm", axis=1, label=lab)   # axis forced to 1 (operation.py:142)
    if kind == "activation":
        m = attrs.get("activation") or "relu"
        return OpSpec("activation", method=m if m in ("tanh", "relu", "sigmoid", "softmax") else "relu", label=lab)
    return None


def parse_combination(node: dict) -> CombSpec | None:
    children = node.get("children") or []
    if not children:
        return None
    c = children[0]
    kind = get_type(c)
    if kind in ("sum", "product"):
        return CombSpec(kind, label=c.get("label", ""))
    if kind == "concat":
        return CombSpec("concat", axis=1, label=c.get("label", ""))   # axis forced to 1 (operation.py:228)
    return None


def parse_output(node: dict) -> OutSpec | None:
    children = node.get("children") or []
    if not children:
        return None
    o = children[0]
    kind = get_type(o)
    lab = o.get("label", "")
    attrs = {get_type(ch): _first_child_type(ch) for ch in o.get("children") or []}
    if kind == "block":
        v = attrs.get("relativeblockindex")
        return OutSpec("block", rel_block_index=int(v) if v else 0, label=lab)
    if kind == "cell":
        v = attrs.get("relativecellindex")
        return OutSpec("cell", rel_cell_index=(int(v) + 1) if v else 1, label=lab)
    return OutSpec("out", label=lab)


def parse_cell(node: dict) -> CellSpec:
    children = list(reversed(node.get("children") or []))
    cell = CellSpec()
    for ch in children:
        if not ch.get("children"):
            continue
        t = get_type(ch)
        if t in ("input1", "input2"):
            el = parse_input(ch)
            if el is not None:
                setattr(cell, t, el)
        elif t in ("operation1", "operation2"):
            el = parse_operation(ch)
            if el is not None:
                setattr(cell, "op1" if t == "operation1" else "op2", el)
        elif t == "combination":
            el = parse_combination(ch)
            if el is not None:
                cell.comb = el
        elif t == "output":
            el = parse_output(ch)
            if el is not None:
                cell.output = el
    return cell


def parse_block(node: dict) -> BlockSpec:
    block = BlockSpec()
    cells = []
    for ch in node.get("children") or []:
        lab = ch.get("label", "")
        t = lab[lab.rfind("_") + 1:]
        if t == "stride":
            v = ch["children"][0]["label"]
            block.set_stride(v[v.rfind("_") + 1:])
        elif t == "features":
            v = ch["children"][0]["label"]
            block.set_features(v[v.rfind("_") + 1:])
        elif ch.get("children"):
            cl = ch["children"][0]["label"]
            ctype = "".join(c for c in cl[cl.rfind("_") + 1:] if not c.isdigit())
            if ctype == "Cell":
                cells.append(parse_cell(ch["children"][0]))
    block.cells = cells  # creation order == the reference's uuid1-ordered sort
    return block


def parse_feature_model(product_tree, name: str | None = None, depth: int = 1, product_features=None,
                        features_label=None) -> ModelSpec:
    """Build a ModelSpec from a product tree, or from a template name (``"lenet5"``, ``"keras"``, ...)."""
    model = ModelSpec(name=name) if name else ModelSpec()
    if product_features:
        model.features = [1 if str(x).isdigit() and int(x) > 0 else 0 for x in product_features]
    if features_label:
        model.features_label = list(features_label)
    if isinstance(product_tree, str):
        from .templates import get_template

        model.blocks = get_template(product_tree)
        return model
    if not product_tree:
        return model
    for _ in range(depth):
        for bd in product_tree:
            bd = copy.deepcopy(bd)
            bd["children"] = list(reversed(bd.get("children") or []))
            model.blocks.append(parse_block(bd))
    return model
