"""Model graph export (reference ``keras.utils.plot_model`` PNG,
``tensorflow_generator.py:356-366``; served by the UI, ``ui/back/main.py:171-173``).

graphviz / pydot are not part of the image, so the graph of a compiled
:class:`~featurenet_amd.ir.compile.CandidateNet` is emitted as

* a JSON node/edge list (machine readable, what the dashboard renders),
* Graphviz DOT text (render elsewhere with ``dot -Tpng``),
* a self-contained SVG drawn here: one row per instruction in program
  (topological) order, skip edges routed on the right.
"""
from __future__ import annotations

import html
import json
from pathlib import Path


def _label(net, kind, arg) -> str:
    if kind in ("module", "head"):
        m = net.mods[arg]
        name = type(m).__name__
        extra = []
        for attr in ("cin", "cout", "kernel", "stride", "padding", "act", "fin", "fout", "kind"):
            v = getattr(m, attr, None)
            if v is not None and not callable(v):
                extra.append(f"{attr}={v}")
        return f"{name}({', '.join(extra)})" if extra else name
    if kind in ("act", "dropout"):
        return f"{kind}({arg})"
    return kind


def graph(net) -> dict:
    nodes, edges = [], []
    for i, (kind, arg, ins) in enumerate(net.prog):
        nodes.append({"id": i, "kind": kind, "label": _label(net, kind, arg)})
        edges += [{"src": j, "dst": i} for j in ins]
    return {"name": getattr(net, "spec_name", ""), "params": getattr(net, "nb_params", None),
            "layers": getattr(net, "nb_layers", None), "nodes": nodes, "edges": edges}


def to_dot(net) -> str:
    g = graph(net)
    lines = [f'digraph "{g["name"] or "model"}" {{', "  node [shape=box, fontname=monospace];"]
    for n in g["nodes"]:
        lines.append(f'  n{n["id"]} [label="{n["label"]}"];')
    for e in g["edges"]:
        lines.append(f'  n{e["src"]} -> n{e["dst"]};')
    lines.append("}")
    return "\n".join(lines) + "\n"


def to_svg(net, row_h: int = 34, width: int = 520) -> str:
    g = graph(net)
    n = len(g["nodes"])
    h = row_h * n + 20
    out = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{width + 120}" height="{h}" font-family="monospace" '
           f'font-size="11">']
    box_w = width - 40
    for e in g["edges"]:
        y1 = 10 + e["src"] * row_h + row_h - 8
        y2 = 10 + e["dst"] * row_h
        if e["dst"] == e["src"] + 1:
            out.append(f'<line x1="{20 + box_w / 2}" y1="{y1}" x2="{20 + box_w / 2}" y2="{y2}" stroke="#555"/>')
        else:   # skip edge: route right of the boxes
            x = 20 + box_w + 10 + 8 * ((e["dst"] - e["src"]) % 10)
            out.append(f'<polyline points="{20 + box_w},{y1 - 10} {x},{y1 - 10} {x},{y2 + 10} {20 + box_w},{y2 + 10}" '
                       f'fill="none" stroke="#c44"/>')
    for nd in g["nodes"]:
        y = 10 + nd["id"] * row_h
        fill = {"module": "#e8f0fe", "head": "#fde8e8", "input": "#e8fde8"}.get(nd["kind"], "#f4f4f4")
        out.append(f'<rect x="20" y="{y}" width="{box_w}" height="{row_h - 8}" rx="4" fill="{fill}" stroke="#333"/>')
        out.append(f'<text x="28" y="{y + row_h / 2}">{html.escape(nd["label"][:80])}</text>')
    out.append("</svg>")
    return "\n".join(out) + "\n"


def export(net, path_stem: str | Path) -> dict:
    """Write ``{stem}.json``, ``{stem}.dot`` and ``{stem}.svg``; returns the paths."""
    stem = str(path_stem)
    paths = {"json": f"{stem}.json", "dot": f"{stem}.dot", "svg": f"{stem}.svg"}
    Path(paths["json"]).write_text(json.dumps(graph(net)))
    Path(paths["dot"]).write_text(to_dot(net))
    Path(paths["svg"]).write_text(to_svg(net))
    return paths


def summary(net) -> str:
    """Keras-style text summary (reference prints ``model.summary()``, ``tensorflow_generator.py:368-379``)."""
    g = graph(net)
    rows = [f"{'#':>4}  {'op':<60} inputs"]
    rows += [f"{n['id']:>4}  {n['label'][:60]:<60} {[e['src'] for e in g['edges'] if e['dst'] == n['id']]}"
             for n in g["nodes"]]
    rows.append(f"params: {g['params']}  layers: {g['layers']}")
    return "\n".join(rows)
