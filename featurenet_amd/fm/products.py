"""PLEDGE ``.pdt`` product files and product trees.

Reference: ``Products_tree.py:6-138`` (``ProductSet``).  File format (also
what :mod:`featurenet_amd.fm.sampler` writes):

    1->Root              header: feature id -> label, one per line
    2->Base
    ...
    1;2;-3;4;...;        one product per line, signed ids (+ selected)

A *product tree* is the nested ``{"label", "id", "children"}`` structure the
architecture parser consumes: a selected feature's parent is the selected
feature whose label is its label up to the last ``_``; only the top-level
``BlockN`` nodes are returned.  ``binary`` mode turns a product into a 0/1
vector ordered by feature id (the genome of the legacy GA and of
``KerasFeatureVector``).
"""
from __future__ import annotations

import re
from pathlib import Path

_FEAT = re.compile(r"^(\d*)->(\w*)")


class ProductSetError(Exception):
    pass


class ProductSet:
    def __init__(self, url: str | Path | None = None, binary_products: bool = False):
        self.features: dict[str, str] = {}
        self.features_reverse: dict[str, str] = {}
        self.products: list[list] = []
        self.binary_products = binary_products
        self.last_products_url = ""
        if url:
            self.load(url)

    # ------------------------------------------------------------------ io
    def load(self, url: str | Path) -> None:
        p = Path(url)
        if not p.is_file():
            raise ProductSetError(f"product file not found: {url}")
        self.last_products_url = str(p)
        self.features, self.features_reverse, self.products = {}, {}, []
        with open(p) as fh:
            for line in fh:
                m = _FEAT.match(line)
                if m and "->" in line:
                    self.features[m.group(1)] = m.group(2)
                    self.features_reverse[m.group(2)] = m.group(1)
                    continue
                toks = line.strip().split(";")
                if toks and toks[-1] == "":
                    toks = toks[:-1]
                if not toks:
                    continue
                if self.binary_products:
                    toks = sorted(toks, key=lambda t: abs(int(t)))
                    toks = [1 if t.isdigit() and int(t) > 0 else 0 for t in toks]
                self.products.append(toks)

    @property
    def nbFeatures(self) -> int:  # noqa: N802 - reference attribute name
        return len(self.features)

    @property
    def nbProducts(self) -> int:  # noqa: N802
        return len(self.products)

    @staticmethod
    def write(path: str | Path, labels: list[str], products: list[list[int]]) -> Path:
        """Write a .pdt: ``labels[i]`` is feature id i+1; products are signed-id lists or 0/1 vectors."""
        p = Path(path)
        with open(p, "w") as fh:
            for i, lab in enumerate(labels):
                fh.write(f"{i + 1}->{lab}\n")
            for prod in products:
                if prod and all(v in (0, 1) for v in prod) and len(prod) == len(labels):
                    ids = [(i + 1) if v else -(i + 1) for i, v in enumerate(prod)]
                else:
                    ids = list(prod)
                fh.write("".join(f"{v};" for v in ids) + "\n")
        return p

    # ------------------------------------------------------------------ trees
    def selected_ids(self, product) -> list[int]:
        if self.binary_products:
            return [i + 1 for i, v in enumerate(product) if int(v) > 0]
        return [abs(int(x)) for x in product if str(x).isdigit() and int(x) >= 0]

    def format_product(self, prd_index: int = 0, original_product=None, include_original: bool = True,
                       sort_features: bool = False):
        original = self.products[prd_index] if not original_product else original_product
        if not original:
            return None
        ids = self.selected_ids(original)
        pos = {self.features[str(x)]: i for i, x in enumerate(ids)}
        nodes = [{"label": self.features[str(x)], "id": x, "children": []} for x in ids]
        for j in range(len(ids) - 1, -1, -1):
            label = nodes[j]["label"]
            cut = label.rfind("_")
            parent = label[:cut] if cut > -1 else ""
            if parent:
                pi = pos.get(parent)
                if pi:  # (index 0 = Root never adopts, as in the reference)
                    nodes[pi]["children"].append(nodes[j])
        blocks = [n for n in nodes if n["label"].startswith("Block") and "_" not in n["label"]]
        if include_original:
            feats = sorted(original, key=lambda k: abs(int(k))) if sort_features else original
            return blocks, feats
        return blocks

    def format_products(self, include_original: bool = True, sort_features: bool = False):
        return [self.format_product(original_product=p, include_original=include_original,
                                    sort_features=sort_features) for p in self.products]

    def light_product(self, prd_index: int = 0, product=None):
        prod = product if product else self.products[prd_index]
        blocks, _ = self.format_product(original_product=prod)

        def light(n):
            n["label"] = n["label"][n["label"].rfind("_"):]
            n["children"] = sorted((light(c) for c in n["children"]), key=lambda c: c["id"])
            return n

        return [light(b) for b in blocks]

    def light_products(self):
        for p in self.products:
            yield self.light_product(product=p)

    @staticmethod
    def filter_leaves(features: dict[str, str], keep_list=None) -> dict[str, str]:
        """Labels worth constraining against (reference behaviour: every label longer than 3 chars)."""
        return {k: v for k, v in features.items() if len(k) > 3}

    def binary_vector(self, product) -> list[int]:
        sel = set(self.selected_ids(product))
        return [1 if i + 1 in sel else 0 for i in range(self.nbFeatures)]

    def enabled_labels(self, product) -> list[str]:
        return [self.features[str(i)] for i in self.selected_ids(product) if str(i) in self.features]
