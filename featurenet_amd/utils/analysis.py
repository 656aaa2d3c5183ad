"""Result analysis: report/evolution plots (SVG) and cross-dataset correlation.

Reference: ``plots/plotter.py`` (accuracy vs time/params, cumulative accuracy
histogram, learning curves, efficiency ``:104-117``, training-time summary
``:120-124``, standard-vs-FeatureNet learning curves ``:128-169``, overfitting
grid ``:174-199``, per-feature accuracy attribution / #features vs accuracy
``:207-297``), ``plots/full_evolution_plotter.py`` (per-epoch
accuracy x robustness Pareto scatter, robustness histogram with a linear fit)
and ``correlation.py`` (Kendall tau / Pearson / Spearman between the MNIST and
CIFAR accuracies of the same products, threshold counts).

matplotlib is not in the image, so charts are written as small standalone
SVG files by :class:`SvgChart`.
"""
from __future__ import annotations

import html
import math
from pathlib import Path

import numpy as np

from .reports import read_population, read_report

PALETTE = ("#1f77b4", "#ff7f0e", "#2ca02c", "#d62728", "#9467bd", "#8c564b", "#e377c2", "#7f7f7f")


class SvgChart:
    def __init__(self, title: str, xlabel: str, ylabel: str, w: int = 640, h: int = 420, logx: bool = False):
        self.title, self.xlabel, self.ylabel, self.w, self.h, self.logx = title, xlabel, ylabel, w, h, logx
        self.series: list = []          # (kind, xs, ys, label)

    def scatter(self, xs, ys, label=""):
        self.series.append(("scatter", np.asarray(xs, float), np.asarray(ys, float), label))
        return self

    def line(self, xs, ys, label=""):
        self.series.append(("line", np.asarray(xs, float), np.asarray(ys, float), label))
        return self

    def bars(self, edges, counts, label=""):
        self.series.append(("bars", np.asarray(edges, float), np.asarray(counts, float), label))
        return self

    def _bounds(self):
        xs = np.concatenate([s[1] for s in self.series]) if self.series else np.zeros(1)
        ys = np.concatenate([s[2] for s in self.series]) if self.series else np.zeros(1)
        if self.logx:
            xs = np.log10(np.maximum(xs, 1e-12))
        x0, x1 = float(np.nanmin(xs)), float(np.nanmax(xs))
        y0, y1 = min(0.0, float(np.nanmin(ys))), float(np.nanmax(ys))
        return x0, (x1 if x1 > x0 else x0 + 1), y0, (y1 if y1 > y0 else y0 + 1)

    def svg(self) -> str:
        L, R, T, B = 60, 20, 30, 45
        x0, x1, y0, y1 = self._bounds()
        pw, ph = self.w - L - R, self.h - T - B

        def X(v):
            v = math.log10(max(v, 1e-12)) if self.logx else v
            return L + (v - x0) / (x1 - x0) * pw

        def Y(v):
            return T + ph - (v - y0) / (y1 - y0) * ph

        out = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{self.w}" height="{self.h}" font-family="sans-serif" '
               f'font-size="11">', f'<text x="{self.w / 2}" y="16" text-anchor="middle" font-size="13">'
               f'{html.escape(self.title)}</text>',
               f'<rect x="{L}" y="{T}" width="{pw}" height="{ph}" fill="none" stroke="#333"/>']
        for i in range(5):
            xv, yv = x0 + (x1 - x0) * i / 4, y0 + (y1 - y0) * i / 4
            lab = f"{10 ** xv:.3g}" if self.logx else f"{xv:.3g}"
            out.append(f'<text x="{L + pw * i / 4}" y="{T + ph + 14}" text-anchor="middle">{lab}</text>')
            out.append(f'<text x="{L - 4}" y="{Y(yv) + 4}" text-anchor="end">{yv:.3g}</text>')
        out.append(f'<text x="{L + pw / 2}" y="{self.h - 8}" text-anchor="middle">{html.escape(self.xlabel)}</text>')
        out.append(f'<text x="14" y="{T + ph / 2}" transform="rotate(-90 14 {T + ph / 2})" text-anchor="middle">'
                   f'{html.escape(self.ylabel)}</text>')
        for k, (kind, xs, ys, label) in enumerate(self.series):
            col = PALETTE[k % len(PALETTE)]
            if kind == "scatter":
                out += [f'<circle cx="{X(a):.1f}" cy="{Y(b):.1f}" r="3" fill="{col}" fill-opacity="0.7"/>'
                        for a, b in zip(xs, ys) if np.isfinite(a) and np.isfinite(b)]
            elif kind == "line":
                pts = " ".join(f"{X(a):.1f},{Y(b):.1f}" for a, b in zip(xs, ys) if np.isfinite(a) and np.isfinite(b))
                out.append(f'<polyline points="{pts}" fill="none" stroke="{col}" stroke-width="1.5"/>')
            else:
                for a, b, c in zip(xs[:-1], xs[1:], ys):
                    out.append(f'<rect x="{X(a):.1f}" y="{Y(c):.1f}" width="{max(X(b) - X(a) - 1, 1):.1f}" '
                               f'height="{Y(y0) - Y(c):.1f}" fill="{col}" fill-opacity="0.6"/>')
            if label:
                out.append(f'<text x="{L + pw - 4}" y="{T + 14 + 13 * k}" text-anchor="end" fill="{col}">'
                           f'{html.escape(label)}</text>')
        out.append("</svg>")
        return "\n".join(out) + "\n"

    def save(self, path: str | Path) -> Path:
        p = Path(path)
        p.write_text(self.svg())
        return p


# --------------------------------------------------------------- report plots
def plot_report(report_path: str | Path, out_dir: str | Path) -> list[Path]:
    """accuracy vs training time, accuracy vs params (log), cumulative accuracy, learning curves."""
    rows = read_report(report_path)
    out = Path(out_dir)
    out.mkdir(parents=True, exist_ok=True)
    acc = [r["accuracy"] for r in rows]
    paths = [SvgChart("accuracy vs training time", "time (s)", "accuracy").scatter([r["time"] for r in rows], acc)
             .save(out / "acc_time.svg"),
             SvgChart("accuracy vs parameters", "params", "accuracy", logx=True)
             .scatter([max(r["params"], 1) for r in rows], acc).save(out / "acc_params.svg")]
    s = np.sort(np.asarray(acc))
    paths.append(SvgChart("cumulative accuracy", "accuracy", "fraction of products")
                 .line(s, np.arange(1, len(s) + 1) / max(len(s), 1)).save(out / "acc_cumulative.svg"))
    lc = SvgChart("learning curves", "epoch", "accuracy")
    for r in rows[:8]:
        for key in ("acc", "val_acc"):
            v = r["history"].get(key)
            if v:
                lc.line(np.arange(1, len(v) + 1), v, f"{r['index']}:{key}")
    paths.append(lc.save(out / "learning_curves.svg"))
    return paths


def plot_evolution(session_dir: str | Path, out_dir: str | Path | None = None) -> list[Path]:
    """Per generation: accuracy x robustness scatter; robustness histogram with a linear fit."""
    sd = Path(session_dir)
    out = Path(out_dir or sd / "plots")
    out.mkdir(parents=True, exist_ok=True)
    paths = []
    gens = sorted(sd.glob("e*.json"), key=lambda p: int(p.stem[1:]) if p.stem[1:].isdigit() else -1)
    pareto = SvgChart("accuracy x robustness per generation", "accuracy", "robustness")
    all_rob = []
    for g in gens:
        if not g.stem[1:].isdigit():
            continue
        recs = [v for _, _, v in read_population(g)]
        a = [float(v[0] or 0) for v in recs]
        r = [float(v[1][2][0] or 0) for v in recs]
        all_rob += r
        pareto.scatter(a, r, g.stem)
    paths.append(pareto.save(out / "pareto.svg"))
    if all_rob:
        counts, edges = np.histogram(all_rob, bins=20)
        h = SvgChart("robustness histogram", "robustness", "count").bars(edges, counts)
        centers = (edges[:-1] + edges[1:]) / 2
        if len(centers) > 1:
            k, b = np.polyfit(centers, counts, 1)
            h.line(centers, k * centers + b, f"fit {k:.3g}x+{b:.3g}")
        paths.append(h.save(out / "robustness_hist.svg"))
    return paths


def efficiency(report_path: str | Path, out_path: str | Path, min_accuracy: float = 0.0) -> Path:
    """Accuracy vs log(parameter count) (reference ``plots/plotter.py:104-117``)."""
    rows = [r for r in read_report(report_path) if r["accuracy"] >= min_accuracy]
    return (SvgChart("efficiency", "log(size)", "accuracy")
            .scatter([math.log(max(r["params"], 1)) for r in rows], [r["accuracy"] for r in rows])
            .save(out_path))


def training_time(report_path: str | Path) -> dict:
    """Sum / median / mean training time of a report (reference ``plots/plotter.py:120-124``)."""
    t = np.asarray([r["time"] for r in read_report(report_path)], float)
    if t.size == 0:
        return {"n": 0, "sum": 0.0, "median": 0.0, "mean": 0.0}
    return {"n": int(t.size), "sum": float(t.sum()), "median": float(np.median(t)), "mean": float(t.mean())}


def _curves(rows, key):
    return [np.asarray(r["history"].get(key, []), float) for r in rows if r["history"].get(key)]


def _mean_curve(curves, n):
    cs = [c[:n] for c in curves if len(c) >= 1]
    if not cs:
        return np.zeros(0)
    m = min(n, min(len(c) for c in cs))
    return np.mean([c[:m] for c in cs], axis=0)


def compare_accuracy(report_path: str | Path, out_path: str | Path, group: int = 10, epochs: int = 150,
                     min_accuracy: float = 0.0) -> Path:
    """Mean learning curves of two run groups: the first ``group`` report lines (the
    hand-written "standard implementation") vs the next ``group`` (the FeatureNet-built
    model); training and test accuracy of each (reference ``plots/plotter.py:128-169``,
    which compares 10 hand-written LeNet-5 runs with 10 ``lenet5``-template runs)."""
    rows = [r for r in read_report(report_path) if r["accuracy"] >= min_accuracy]
    std, ours = rows[:group], rows[group:2 * group]
    ch = SvgChart("standard vs FeatureNet implementation", "iteration", "accuracy")
    for name, grp in (("standard", std), ("ours", ours)):
        for key, lab in (("acc", "training"), ("val_acc", "test")):
            y = _mean_curve(_curves(grp, key), epochs)
            if y.size:
                ch.line(np.arange(y.size), y, f"{name} {lab}")
    return ch.save(out_path)


def overfitting(report_path: str | Path, out_path: str | Path, min_accuracy: float = 0.0, cols: int = 3) -> Path:
    """One panel per architecture: training vs test accuracy per iteration, titled with the
    final accuracy and the parameter count (reference ``plots/plotter.py:174-199``)."""
    rows = [r for r in read_report(report_path) if r["accuracy"] >= min_accuracy]
    pw, ph = 320, 220
    nrow = max(1, math.ceil(len(rows) / cols))
    parts = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{cols * pw}" height="{nrow * ph + 24}" '
             f'font-family="sans-serif" font-size="10">',
             f'<text x="{cols * pw / 2}" y="16" text-anchor="middle" font-size="12">'
             f'<tspan fill="{PALETTE[0]}">training accuracy</tspan>  <tspan fill="{PALETTE[3]}">test accuracy'
             f'</tspan></text>']
    for i, r in enumerate(rows):
        ch = SvgChart(f"architecture {r['index']} {r['accuracy'] * 100:.2f}% {r['params'] / 1e6:.2f}M",
                      "iteration", "accuracy", w=pw, h=ph)
        for key in ("acc", "val_acc"):
            v = r["history"].get(key)
            if v:
                ch.scatter(np.arange(len(v)), v)
        if not ch.series:
            ch.scatter([0], [r["accuracy"]])
        body = ch.svg().split("\n", 1)[1].rsplit("</svg>", 1)[0]
        x, y = (i % cols) * pw, (i // cols) * ph + 24
        parts.append(f'<g transform="translate({x},{y})">{body}</g>')
    parts.append("</svg>")
    p = Path(out_path)
    p.write_text("\n".join(parts) + "\n")
    return p


def feature_attribution(report_path: str | Path, pdt_path: str | Path, top: int = 10) -> dict:
    """Per-feature accuracy attribution (reference ``plots/plotter.py:207-297``): for every
    feature enabled in some product, the average / max / min accuracy of the products that
    enable it; leaf features (labels with more than 4 ``_``-separated parts) ranked by
    average accuracy; and the enabled-feature count of every product."""
    from ..fm.products import ProductSet

    rows = read_report(report_path)
    acc = {r["index"]: r["accuracy"] for r in rows}
    ps = ProductSet(pdt_path)
    per_feat: dict[int, list[float]] = {}
    counts, accs = [], []
    for i, prod in enumerate(ps.products):
        a = acc.get(i, acc.get(i + 1))
        if a is None:
            continue
        ids = ps.selected_ids(prod)
        counts.append(len(ids))
        accs.append(a)
        for f in ids:
            per_feat.setdefault(f, []).append(a)
    stats = {ps.features[str(f)]: {"avg": float(np.mean(v)), "max": float(np.max(v)), "min": float(np.min(v)),
                                   "n": len(v)} for f, v in per_feat.items() if str(f) in ps.features}
    leaves = {k: v for k, v in stats.items() if len(k.split("_")) > 4}
    ranked = sorted(leaves.items(), key=lambda kv: kv[1]["avg"])
    return {"features": stats, "lowest": ranked[:top], "highest": ranked[::-1][:top],
            "n_features_per_product": counts, "accuracy": accs}


def plot_feature_attribution(report_path: str | Path, pdt_path: str | Path, out_dir: str | Path,
                             top: int = 10) -> list[Path]:
    """Bars of the lowest / highest average-accuracy leaf features (accuracy squared, as the
    reference plots it), #enabled features vs accuracy, and max / average accuracy per leaf."""
    res = feature_attribution(report_path, pdt_path, top)
    out = Path(out_dir)
    out.mkdir(parents=True, exist_ok=True)
    paths = []
    for name, items in (("lowest", res["lowest"]), ("highest", res["highest"])):
        ch = SvgChart(f"features with {name} average accuracy", "rank", "accuracy^2")
        if items:
            ch.bars(np.arange(len(items) + 1), [v["avg"] ** 2 for _, v in items])
        paths.append(ch.save(out / f"features_{name}.svg"))
        (out / f"features_{name}.txt").write_text("".join(f"{k}\t{v['avg']:.4f}\t{v['n']}\n" for k, v in items))
    paths.append(SvgChart("accuracy vs enabled features", "number of enabled features", "accuracy")
                 .scatter(res["n_features_per_product"], res["accuracy"]).save(out / "features_count.svg"))
    leaves = sorted((v for k, v in res["features"].items() if len(k.split("_")) > 4), key=lambda v: v["avg"])
    ch = SvgChart("accuracy of the configurations of each leaf feature", "leaf feature", "accuracy")
    if leaves:
        ch.scatter(np.arange(len(leaves)), [v["max"] for v in leaves], "max")
        ch.scatter(np.arange(len(leaves)), [v["avg"] for v in leaves], "average")
    paths.append(ch.save(out / "features_leaves.svg"))
    return paths


# --------------------------------------------------------------- correlation
def correlation(acc_a, acc_b, thresholds=(0.5, 0.7, 0.9)) -> dict:
    """Kendall tau / Pearson / Spearman between two accuracy lists of the same products."""
    from scipy import stats

    a, b = np.asarray(acc_a, float), np.asarray(acc_b, float)
    n = min(len(a), len(b))
    a, b = a[:n], b[:n]
    res = {"n": n, "kendall": stats.kendalltau(a, b)[0], "pearson": stats.pearsonr(a, b)[0],
           "spearman": stats.spearmanr(a, b)[0]}
    res["thresholds"] = {t: {"a": int((a >= t).sum()), "b": int((b >= t).sum()), "both": int(((a >= t) & (b >= t)).sum())}
                         for t in thresholds}
    return res


def correlate_reports(report_a: str | Path, report_b: str | Path, **kw) -> dict:
    ra = {r["index"]: r["accuracy"] for r in read_report(report_a)}
    rb = {r["index"]: r["accuracy"] for r in read_report(report_b)}
    common = sorted(set(ra) & set(rb))
    return correlation([ra[i] for i in common], [rb[i] for i in common], **kw)
