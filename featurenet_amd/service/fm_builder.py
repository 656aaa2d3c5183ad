"""Cell feature-model builder behind the dashboard's "FM builder" page.

Reference: the React page ``ui/src/pages/fm.js:112-118`` shows a checkable tree
of cell features (catalogue ``ui/src/util.js:1-210``: two inputs with
convolution / pooling / dense / identity / zeros alternatives and their
attribute values, two operations, the combination and the output routing)
and ``buildTree`` (``ui/src/util.js:240-262``) turns the checked keys into a
SPLOT feature model (the ``Block[k]`` / ``Block[k]_Element[i]`` template of
``defaultXML``, ``ui/src/util.js:214-238``) that the user downloads as
``fm.xml`` and later feeds to the extender / sampler.

Differences from the reference, all deliberate:

* keys are unique paths (``input1/convolution/kernel/3x1``); the reference
  reuses ``1x1-kernel...`` for three kernel entries and lists ``Identity``
  twice, so those checkboxes toggle together;
* the emitted tree is indented by depth, as SPLOT requires (the reference's
  ``iterNode`` emits every feature at column 0, which no SPLOT parser reads as a
  tree), in the shape of the reference template ``main_1block_nas.xml`` (choices
  are mandatory features holding a ``[1,1]`` group of their checked
  alternatives; an alternative's attributes are mandatory choices below it),
  with the labels ``iterNode`` gives them;
* constraints that name an unchecked cell feature are dropped (the reference
  always emits all seven, so e.g. C7 names ``Input1_Zeros`` even when Zeros is
  unchecked);
* the result is checked by parsing it with :mod:`featurenet_amd.fm.splot`.
"""
from __future__ import annotations

from ..fm.space import CELL

_RELU_ONLY = {"sigmoid", "tanh", "softmax"}


def _leaves(values, disabled=()):
    return [{"title": v, "disabled": v in disabled} for v in values]


def _input(idx: int) -> dict:
    return {"title": f"Input{idx}", "children": [
        {"title": "Convolution", "children": [
            {"title": "kernel", "children": _leaves(["1x1", "3x1", "1x3", "3x3", "1x5", "5x1", "5x5", "7x1", "1x7"])},
            {"title": "type", "children": _leaves(["normal", "separable", "depthwise"])},
            {"title": "activation", "children": _leaves(["relu", "sigmoid", "tanh", "softmax"], _RELU_ONLY)},
            {"title": "padding", "children": _leaves(["same", "valid"])},
            {"title": "features", "children": _leaves(["16", "32", "64", "128", "256", "512", "1024", "2048"],
                                                      {"256", "512", "1024", "2048"})},
            {"title": "stride", "children": _leaves(["1x1", "2x2", "3x3"], {"1x1", "3x3"})},
        ]},
        {"title": "Identity"},
        {"title": "Recurrence"},
        {"title": "Zeros"},
        {"title": "Pooling", "children": [
            {"title": "kernel", "children": _leaves(["1x1", "2x2", "3x3"])},
            {"title": "type", "children": _leaves(["max", "average", "dilated", "global"])},
            {"title": "padding", "children": _leaves(["same", "valid"])},
            {"title": "stride", "children": _leaves(["1x1", "2x2", "3x3"], {"1x1", "3x3"})},
        ]},
        {"title": "Dense", "children": [
            {"title": "features", "children": _leaves(["8", "16", "32", "64", "96", "256", "512", "1024", "2048"],
                                                      {"256", "512", "1024", "2048"})},
            {"title": "activation", "children": _leaves(["relu", "sigmoid", "tanh", "softmax"], _RELU_ONLY)},
        ]},
    ]}


def _operation(idx: int) -> dict:
    return {"title": f"Operation{idx}", "children": [
        {"title": "Void"},
        {"title": "BatchNormalization"},
        {"title": "Flatten"},
        {"title": "Activation", "children": _leaves(["relu", "sigmoid", "tanh", "softmax"], _RELU_ONLY)},
        {"title": "Padding", "children": [{"title": "fillSize", "children": _leaves(["0x1", "1x0", "1x1", "3x3"])}]},
        {"title": "Dropout", "children": [{"title": "value", "children": _leaves(["0", "2", "5", "7"])}]},
    ]}


def _with_keys(node: dict, prefix: str = "") -> dict:
    key = f"{prefix}/{node['title'].lower()}" if prefix else node["title"].lower()
    out = {"title": node["title"], "key": key, "disabled": bool(node.get("disabled", False))}
    if node.get("children"):
        out["children"] = [_with_keys(c, key) for c in node["children"]]
    return out


def catalogue() -> list[dict]:
    """The checkable cell-feature tree (titles, unique keys, disabled flags)."""
    cell = {"title": "Cell", "children": [
        _input(1), _input(2), _operation(1), _operation(2),
        {"title": "Combination", "children": [{"title": "Sum"}, {"title": "Concat"}]},
        {"title": "Output", "children": [
            {"title": "Block"},
            {"title": "Cell", "children": [{"title": "relativeCellIndex", "children": _leaves(["0", "1", "2"])}]},
        ]},
    ]}
    return [_with_keys(cell)]


HEADER = (":r Root(Root)", 0), (":m Base(Base)", 1), (":m Training(Training)", 2), \
    (":m Architecture(Architecture)", 3), (":m Input(Input)", 4), (":m Output(Output)", 4), \
    (":o Block[k](Block[k])", 4), (":m Block[k]_stride(Block[k]_stride)", 5), (":g [1,1]", 6), \
    (": Block[k]_stride_2x2(Block[k]_stride_2x2)", 7), (": Block[k]_stride_1x1(Block[k]_stride_1x1)", 7), \
    (":m Block[k]_features(Block[k]_features)", 5), (":g [1,1]", 6)
BLOCK_FEATURES = ("800", "400", "200", "100", "50", "25")
CONSTRAINTS = (
    "~Architecture  or  Block1",
    "~Block[k+1]  or  Block[k]",
    "~Block[k]_Element[i+1]  or  Block[k]_Element[i]",
    f"~{CELL}_Output_Block  or  Block[k+1]",
    f"~{CELL}_Output_Block  or  ~Block[k]_Element[i+1]",
    f"~{CELL}_Output_Cell  or  Block[k]_Element[i+1]",
    f"~Architecture  or  ~{CELL}_Input1_Zeros",
)


def build_fm(checked: list[str]) -> str:
    """SPLOT XML of the cell template restricted to the checked catalogue keys."""
    sel = set(checked)
    lines = [("\t" * d) + t for t, d in HEADER]
    lines += [("\t" * 7) + f": Block[k]_features_{v}(Block[k]_features_{v})" for v in BLOCK_FEATURES]
    lines += [("\t" * 5) + ":o Block[k]_Element[i](Block[k]_Element[i])", ("\t" * 6) + f":o {CELL}({CELL})"]

    # SPLOT shape of the reference template (main_1block_nas.xml): a choice (Input1,
    # Convolution_kernel, ...) is a mandatory feature holding a [1,1] group of its
    # alternatives; an alternative with attributes (Convolution) is a group member whose
    # attributes are mandatory choices one level down; an alternative with bare values
    # (Activation -> relu) holds its own [1,1] group
    def choice(node: dict, label: str, depth: int):
        lab = f"{label}_{node['title']}"
        lines.append(("\t" * depth) + f":m {lab}({lab})")
        kids = [c for c in node.get("children", []) if c["key"] in sel]
        if kids:
            lines.append(("\t" * (depth + 1)) + ":g [1,1]")
            for c in kids:
                member(c, lab, depth + 2)

    def member(node: dict, label: str, depth: int):
        lab = f"{label}_{node['title']}"
        lines.append(("\t" * depth) + f": {lab}({lab})")
        kids = [c for c in node.get("children", []) if c["key"] in sel]
        if kids and all(not c.get("children") for c in node["children"]):
            lines.append(("\t" * (depth + 1)) + ":g [1,1]")
            for c in kids:
                lines.append(("\t" * (depth + 2)) + f": {lab}_{c['title']}({lab}_{c['title']})")
        else:
            for c in kids:
                choice(c, lab, depth + 1)

    for child in catalogue()[0]["children"]:
        if child["key"] in sel:
            choice(child, CELL, 7)
    names = {ln.strip().split(" ", 1)[1].split("(", 1)[0] for ln in lines if " " in ln.strip()}
    keep = [c for c in CONSTRAINTS
            if all(lit.lstrip("~") in names for lit in c.split("  or  ") if CELL in lit)]
    cons = "\n".join(f"C{i + 1}:{c}" for i, c in enumerate(keep))
    return ('<?xml version="1.0" encoding="UTF-8" standalone="no"?>\n<feature_model name="FeatureNet model">\n'
            "<feature_tree>\n" + "\n".join(lines) + "\n</feature_tree>\n<constraints>\n" + cons +
            "\n</constraints>\n</feature_model>\n")
