"""Programmatic NAS search-space (feature model) builder.

The reference ships its search space as a hand-written FeatureIDE/SPLOT file
(``main_1block_nas.xml``): one block ``Block[k]`` holding one cell element
``Block[k]_Element[i]`` whose sub-features choose the two inputs, two
operations, the combination and the output routing.  The extender
(:mod:`featurenet_amd.fm.extend`) then instantiates ``[k]``/``[i]`` into B x C.

Here the same space is *described* as data (:class:`SearchSpace`) and rendered
to SPLOT XML, so it can be customised (other kernel sets, activations,
dropout values, ...) without editing XML by hand.  ``SearchSpace()`` with the
defaults renders the reference template byte-for-byte (tested), which keeps
the extender goldens and PLEDGE product files interchangeable.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from pathlib import Path

CELL = "Block[k]_Element[i]_Cell"


@dataclass
class SearchSpace:
    input1_kernels: tuple = ("1x1", "3x1", "1x3", "3x3", "1x5", "5x1", "5x5", "1x7", "7x1")
    input2_kernels: tuple = ("1x1", "2x2", "3x1", "1x3", "3x3", "1x5", "5x1")
    conv_types: tuple = ("normal", "separable", "depthwise")
    paddings: tuple = ("same",)
    activations: tuple = ("relu",)
    input_kinds: tuple = ("Convolution", "Identity", "Zeros")
    operations: tuple = ("Void", "BatchNormalization", "Dropout")
    dropout_values: tuple = ("5", "0")
    combinations: tuple = ("Concat", "Sum")
    cell_indices: tuple = ("0", "1", "2")
    extra_constraints: list = field(default_factory=list)

    # ----------------------------------------------------------------- tree
    def _feature_lines(self) -> list[tuple[int, str, str]]:
        """(depth, kind marker, name) rows in SPLOT order."""
        rows: list[tuple[int, str, str]] = [(0, ":r", "Root"), (1, ":m", "Base"), (2, ":m", "Training"),
                                            (3, ":m", "Architecture"), (4, ":m", "Input"), (4, ":m", "Output"),
                                            (4, ":o", "Block[k]"), (5, ":o", "Block[k]_Element[i]"),
                                            (6, ":o", CELL)]

        def group(depth, names):
            rows.append((depth, ":g", "[1,1]"))
            for n in names:
                rows.append((depth + 1, ":", n))

        def attr_group(depth, base, attr, values):
            rows.append((depth, ":m", f"{base}_{attr}"))
            group(depth + 1, [f"{base}_{attr}_{v}" for v in values])

        for idx, kernels in ((1, self.input1_kernels), (2, self.input2_kernels)):
            inp = f"{CELL}_Input{idx}"
            rows.append((7, ":m", inp))
            rows.append((8, ":g", "[1,1]"))
            for kind in self.input_kinds:
                rows.append((9, ":", f"{inp}_{kind}"))
                if kind == "Convolution":
                    conv = f"{inp}_Convolution"
                    attr_group(10, conv, "kernel", kernels)
                    attr_group(10, conv, "type", self.conv_types)
                    attr_group(10, conv, "padding", self.paddings)
                    attr_group(10, conv, "activation", self.activations)
        for idx in (1, 2):
            op = f"{CELL}_Operation{idx}"
            rows.append((7, ":m", op))
            rows.append((8, ":g", "[1,1]"))
            for kind in self.operations:
                rows.append((9, ":", f"{op}_{kind}"))
                if kind == "Dropout" and self.dropout_values:
                    rows.append((10, ":o", f"{op}_Dropout_value"))
                    group(11, [f"{op}_Dropout_value_{v}" for v in self.dropout_values])
        rows.append((7, ":m", f"{CELL}_Combination"))
        group(8, [f"{CELL}_Combination_{c}" for c in self.combinations])
        out = f"{CELL}_Output"
        rows.append((7, ":m", out))
        rows.append((8, ":g", "[1,1]"))
        rows.append((9, ":", f"{out}_Block"))
        rows.append((9, ":", f"{out}_Cell"))
        if self.cell_indices:
            rows.append((10, ":o", f"{out}_Cell_relativeCellIndex"))
            group(11, [f"{out}_Cell_relativeCellIndex_{v}" for v in self.cell_indices])
        return rows

    def tree_text(self) -> str:
        lines = []
        for depth, kind, name in self._feature_lines():
            body = name if kind == ":g" else f"{name}({name})"
            lines.append("\t" * depth + f"{kind} {body}")
        return "\n" + "\n".join(lines) + "\n"

    # ----------------------------------------------------------- constraints
    def constraints(self) -> list[str]:
        cons = ["~Architecture  or  Block1",
                "~Block[k+1]  or  Block[k]",
                "~Block[k]_Element[i+1]  or  Block[k]_Element[i]",
                f"~{CELL}_Output_Block  or  Block[k+1]",
                f"~{CELL}_Output_Block  or  ~Block[k]_Element[i+1]",
                f"~{CELL}_Output_Cell  or  Block[k]_Element[i+1]"]
        if "Zeros" in self.input_kinds:
            cons.append(f"~Architecture  or  ~{CELL}_Input1_Zeros")    # input1 may never be Zeros
        return cons + list(self.extra_constraints)

    def constraints_text(self) -> str:
        return "\n" + "".join(f"C{i + 1}:{c}\n" for i, c in enumerate(self.constraints())) + "\n"

    def xml(self) -> str:
        return ('<?xml version="1.0" encoding="UTF-8" standalone="no"?>\n'
                '<feature_model name="FeatureIDE model">\n'
                f"    <feature_tree>{self.tree_text()}</feature_tree>\n"
                f"    <constraints>{self.constraints_text()}</constraints>\n"
                "</feature_model>\n")

    def write(self, path: str | Path) -> Path:
        p = Path(path)
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(self.xml())
        return p


def default_template(path: str | Path) -> Path:
    """Write the default 1-block / 1-cell NAS template (the reference search space)."""
    return SearchSpace().write(path)
