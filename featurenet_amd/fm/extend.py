"""Template instantiation of a one-block/one-cell feature model to B blocks x C cells.

Reference: ``extender.py:3-62`` (``generate_featuretree``).  The template FM
holds a single block subtree labelled with the placeholder ``[k]`` and a
single cell subtree labelled ``[i]``; constraints may mention ``[k]``,
``[k+1]``, ``[i]``, ``[i+1]``.  Expansion rules (kept identical so the output
is byte-for-byte the reference's ``nas_1_1_10.xml`` for (1, 1)):

* the cell subtree (from ``:o Block[k]_Element[i]`` to the end of the tree
  text) is repeated ``nb_cells`` times with ``[i] -> 1..C``, joined by five
  tabs; then the block subtree (from ``:o Block[k](Block[k])``) is repeated
  ``nb_blocks`` times with ``[k] -> 1..B``, joined by four tabs;
* constraints without ``[k]`` are kept verbatim; constraints whose name
  contains ``CLC`` are dropped; the others are instantiated for every block
  (and every cell when they mention ``[i]``), skipping the ``[k+1]`` /
  ``[i+1]`` instances that would point past the last block / cell;
* instantiated constraints are renumbered ``C<n>`` continuing after the kept
  ones.

The optional per-block ``stride`` / ``features`` subtrees of
``main_1block_nas_blockfeatures.xml`` (reference ``ui/src/util.js:196-238``)
are supported through ``block_features=True``.
"""
from __future__ import annotations

import xml.etree.ElementTree as ET
from pathlib import Path

CELL_ANCHOR = ":o Block[k]_Element[i]"
BLOCK_ANCHOR = ":o Block[k](Block[k])"

BLOCK_FEATURES_TEMPLATE = (
    ":m Block[k]_stride(Block[k]_stride)\n"
    "\t\t\t\t\t\t:g [1,1]\n"
    "\t\t\t\t\t\t\t: Block[k]_stride_2x2(Block[k]_stride_2x2)\n"
    "\t\t\t\t\t\t\t: Block[k]_stride_1x1(Block[k]_stride_1x1)\n"
    "\t\t\t\t\t:m Block[k]_features(Block[k]_features)\n"
    "\t\t\t\t\t\t:g [1,1]\n"
    + "".join(f"\t\t\t\t\t\t\t: Block[k]_features_{v}(Block[k]_features_{v})\n" for v in (800, 400, 200, 100, 50, 25))
    + "\t\t\t\t\t"
)


def expand_tree_text(text: str, nb_cells: int, nb_blocks: int, block_features: bool = False) -> str:
    ci = text.find(CELL_ANCHOR)
    if ci < 0:
        raise ValueError("template feature tree has no cell anchor " + CELL_ANCHOR)
    cell = text[ci:]
    text = text[:ci] + "\t\t\t\t\t".join(cell.replace("[i]", str(i + 1)) for i in range(nb_cells))
    bi = text.find(BLOCK_ANCHOR)
    if bi < 0:
        raise ValueError("template feature tree has no block anchor " + BLOCK_ANCHOR)
    block = text[bi:]
    if block_features:
        # insert the per-block stride/features subtrees right after the block line
        nl = block.find("\n") + 1
        head, tail = block[:nl], block[nl:]
        block = head + "\t\t\t\t\t" + BLOCK_FEATURES_TEMPLATE + tail.lstrip("\t")
    return text[:bi] + "\t\t\t\t".join(block.replace("[k]", str(k + 1)) for k in range(nb_blocks))


def expand_constraints_text(text: str, nb_cells: int, nb_blocks: int) -> str:
    out = ""
    cid = 1
    for line in text.split("\n"):
        parts = line.split(":")
        if len(parts) < 2:
            continue
        name, body = parts[0], parts[1]
        if "[k]" not in body:
            out += "\n" + line
            cid += 1
            continue
        if "CLC" in name:
            continue
        for k in range(nb_blocks):
            if "[k+1]" in body and k + 1 == nb_blocks:
                continue
            kb = body.replace("[k]", str(k + 1)).replace("[k+1]", str(k + 2))
            if "[i]" not in body:
                out += f"\nC{cid}:{kb}"
                cid += 1
                continue
            for i in range(nb_cells):
                if "[i+1]" in body and i + 1 == nb_cells:
                    continue
                out += f"\nC{cid}:" + kb.replace("[i]", str(i + 1)).replace("[i+1]", str(i + 2))
                cid += 1
    return out + "\n"


def generate_featuretree(input_file: str | Path, output_file: str | Path, nb_cells: int, nb_blocks: int,
                         block_features: bool = False) -> Path:
    """Expand ``input_file`` to ``nb_blocks`` x ``nb_cells`` and write ``output_file``."""
    tree = ET.parse(str(input_file))
    root = tree.getroot()
    ft, cs = list(root)[0], list(root)[1]
    ft.text = expand_tree_text(ft.text, nb_cells, nb_blocks, block_features)
    cs.text = expand_constraints_text(cs.text, nb_cells, nb_blocks)
    tree.write(str(output_file), encoding="UTF-8", xml_declaration=True)
    return Path(output_file)
