"""SPLOT feature models embedded in FeatureIDE-style XML.

Reference: the search-space files ``main_1block_nas.xml`` / ``nas_*.xml``
(``<feature_tree>`` holds SPLOT text, ``<constraints>`` holds CNF clauses
``Cn:lit or lit``).  SPLOT line syntax (indentation = depth, tabs):

    :r Name(Id)      root
    :m Name(Id)      mandatory child
    :o Name(Id)      optional child
    :g [a,b]         feature group with cardinality [a,b] (b may be *)
    : Name(Id)       member of the enclosing group

This module parses the text into :class:`Feature` nodes and lowers the whole
model (tree semantics + cross-tree constraints) to CNF over 1-based variable
ids, which the native sampler (``csrc/runtime/sampler.cpp``) and the
pure-Python fallback solver consume.
"""
from __future__ import annotations

import re
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field
from pathlib import Path

_LINE = re.compile(r"^(\t*)\s*:(r|m|o|g)?\s*(.*)$")
_NAMED = re.compile(r"^([^()\s]+)\s*\(([^()]*)\)\s*$")
_CARD = re.compile(r"^\[\s*(\d+)\s*,\s*(\d+|\*)\s*\]$")


@dataclass
class Feature:
    name: str
    kind: str                     # "root" | "mandatory" | "optional" | "member"
    children: list["Feature"] = field(default_factory=list)
    groups: list[tuple[int, int, list["Feature"]]] = field(default_factory=list)  # (min, max, members)
    parent: "Feature | None" = None

    def walk(self):
        yield self
        for c in self.children:
            yield from c.walk()
        for _, _, ms in self.groups:
            for m in ms:
                yield from m.walk()

    def all_children(self) -> list["Feature"]:
        out = list(self.children)
        for _, _, ms in self.groups:
            out.extend(ms)
        return out


@dataclass
class FeatureModel:
    root: Feature
    constraints: list[list[tuple[str, bool]]]   # clauses of (feature name, positive)
    constraint_names: list[str] = field(default_factory=list)

    # ----------------------------------------------------------------- queries
    def features(self) -> list[Feature]:
        return list(self.root.walk())

    def names(self) -> list[str]:
        return [f.name for f in self.root.walk()]

    def index(self) -> dict[str, int]:
        """name -> 1-based variable id (pre-order, matching PLEDGE's numbering)."""
        return {n: i + 1 for i, n in enumerate(self.names())}

    # ----------------------------------------------------------------- CNF
    def to_cnf(self) -> tuple[int, list[list[int]]]:
        idx = self.index()
        clauses: list[list[int]] = [[idx[self.root.name]]]
        for f in self.root.walk():
            v = idx[f.name]
            for c in f.children:
                cv = idx[c.name]
                clauses.append([-cv, v])                 # child -> parent
                if c.kind == "mandatory":
                    clauses.append([-v, cv])             # parent -> mandatory child
            for lo, hi, ms in f.groups:
                mv = [idx[m.name] for m in ms]
                for m in mv:
                    clauses.append([-m, v])              # member -> parent
                if lo >= 1:
                    clauses.append([-v] + mv)            # parent -> at least one
                if hi == 1:
                    for i in range(len(mv)):             # at most one
                        for j in range(i + 1, len(mv)):
                            clauses.append([-mv[i], -mv[j]])
        for cl in self.constraints:
            lits = []
            for name, pos in cl:
                if name not in idx:
                    raise KeyError(f"constraint references unknown feature {name!r}")
                lits.append(idx[name] if pos else -idx[name])
            clauses.append(lits)
        return len(idx), clauses

    def is_valid(self, selected: set[str]) -> bool:
        idx = self.index()
        sel = {idx[n] for n in selected}
        _, clauses = self.to_cnf()
        return all(any((l > 0 and l in sel) or (l < 0 and -l not in sel) for l in cl) for cl in clauses)


def parse_tree_text(text: str) -> Feature:
    root: Feature | None = None
    # stack of (depth, node-or-group-marker)
    stack: list[tuple[int, object]] = []
    for raw in text.splitlines():
        if not raw.strip():
            continue
        m = _LINE.match(raw)
        if not m:
            continue
        depth = len(m.group(1))
        tag = m.group(2)
        rest = m.group(3).strip()
        while stack and stack[-1][0] >= depth:
            stack.pop()
        parent = stack[-1][1] if stack else None
        if tag == "g":
            cm = _CARD.match(rest)
            lo, hi = (1, 1) if not cm else (int(cm.group(1)), -1 if cm.group(2) == "*" else int(cm.group(2)))
            if not isinstance(parent, Feature):
                raise ValueError(f"group without parent feature: {raw!r}")
            grp = (lo, hi, [])
            parent.groups.append(grp)
            stack.append((depth, grp))
            continue
        nm = _NAMED.match(rest)
        name = nm.group(1) if nm else rest.split()[0]
        if tag == "r":
            node = Feature(name, "root")
            root = node
        elif tag in ("m", "o"):
            node = Feature(name, "mandatory" if tag == "m" else "optional")
            if not isinstance(parent, Feature):
                raise ValueError(f"feature {name!r} has no parent")
            node.parent = parent
            parent.children.append(node)
        else:  # group member
            node = Feature(name, "member")
            if not isinstance(parent, tuple):
                raise ValueError(f"group member {name!r} outside a group")
            owner = stack[-2][1] if len(stack) >= 2 else None
            node.parent = owner if isinstance(owner, Feature) else None
            parent[2].append(node)
        stack.append((depth, node))
    if root is None:
        raise ValueError("feature tree has no :r root")
    return root


def parse_constraints_text(text: str) -> tuple[list[list[tuple[str, bool]]], list[str]]:
    clauses, names = [], []
    for line in (text or "").splitlines():
        if ":" not in line:
            continue
        name, body = line.split(":", 1)
        lits = []
        for tok in body.split(" or "):
            tok = tok.strip()
            if not tok:
                continue
            neg = tok.startswith("~")
            lits.append((tok[1:].strip() if neg else tok, not neg))
        if lits:
            clauses.append(lits)
            names.append(name.strip())
    return clauses, names


def load(path: str | Path) -> FeatureModel:
    tree = ET.parse(str(path))
    root = tree.getroot()
    ft = root.find("feature_tree")
    cs = root.find("constraints")
    froot = parse_tree_text(ft.text if ft is not None else "")
    clauses, names = parse_constraints_text(cs.text if cs is not None else "")
    return FeatureModel(froot, clauses, names)


def loads(xml_text: str) -> FeatureModel:
    root = ET.fromstring(xml_text)
    ft = root.find("feature_tree")
    cs = root.find("constraints")
    froot = parse_tree_text(ft.text if ft is not None else "")
    clauses, names = parse_constraints_text(cs.text if cs is not None else "")
    return FeatureModel(froot, clauses, names)


def to_xml(model: FeatureModel) -> str:
    """Serialise back to FeatureIDE/SPLOT XML (round-trips through :func:`loads`)."""
    lines = []

    def emit(f: Feature, depth: int):
        tag = {"root": ":r", "mandatory": ":m", "optional": ":o", "member": ":"}[f.kind]
        lines.append("\t" * depth + f"{tag} {f.name}({f.name})")
        for c in f.children:
            emit(c, depth + 1)
        for lo, hi, ms in f.groups:
            lines.append("\t" * (depth + 1) + f":g [{lo},{'*' if hi < 0 else hi}]")
            for m in ms:
                emit(m, depth + 2)

    emit(model.root, 0)
    cons = []
    for i, cl in enumerate(model.constraints):
        body = "  or  ".join(("" if pos else "~") + n for n, pos in cl)
        cons.append(f"C{i + 1}:{body}")
    return ('<?xml version="1.0" encoding="UTF-8" standalone="no"?>\n<feature_model name="FeatureIDE model">\n'
            "    <feature_tree>\n" + "\n".join(lines) + "\n</feature_tree>\n    <constraints>\n" + "\n".join(cons)
            + "\n</constraints>\n</feature_model>\n")
