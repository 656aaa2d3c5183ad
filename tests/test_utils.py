"""Reports, events, graph export, plots and correlation utilities."""
import json

import numpy as np

from featurenet_amd.utils import analysis
from featurenet_amd.utils.events import EventLog, read_events
from featurenet_amd.utils.reports import (KerasFeatureVector, append_population, read_population, read_report,
                                          report_line)


def test_report_line_roundtrip(tmp_path):
    p = tmp_path / "r.txt"
    with open(p, "w") as f:
        for i in range(5):
            f.write(report_line(i, 0.5 + 0.1 * i, False, 10.0 + i, 1000 * (i + 1), 0, {"acc": [0.1, 0.2],
                                                                                     "val_acc": [0.15, 0.25]}))
    rows = read_report(p)
    assert [r["index"] for r in rows] == list(range(5))
    assert rows[2]["accuracy"] == 0.7 and rows[0]["history"]["val_acc"] == [0.15, 0.25]
    paths = analysis.plot_report(p, tmp_path / "plots")
    assert all(x.read_text().startswith("<svg") for x in paths)


def test_population_log_and_evolution_plot(tmp_path):
    class S:
        def __init__(self, i):
            self.name, self.accuracy, self.robustness_score = f"m{i}", 0.1 * i, 0.05 * i
            self.blocks, self.nb_layers, self.nb_params, self.nb_flops = [], 3, 100, 10
            self.clever_score = self.fgsm_score = self.pgd_score = self.cw_score = 0
            self.metrics, self.features = [], [1, 0]

    for g in (1, 2):
        append_population(tmp_path / f"e{g}.json", [S(i) for i in range(4)])
    recs = read_population(tmp_path / "e1.json")
    assert len(recs) == 4 and KerasFeatureVector.from_vector(recs[3][2]).accuracy == 0.30000000000000004
    paths = analysis.plot_evolution(tmp_path)
    assert len(paths) == 2


def test_correlation_identical_and_reversed():
    a = np.linspace(0.1, 0.9, 9)
    c = analysis.correlation(a, a)
    assert abs(c["kendall"] - 1) < 1e-9 and abs(c["spearman"] - 1) < 1e-9
    c2 = analysis.correlation(a, a[::-1])
    assert abs(c2["pearson"] + 1) < 1e-9
    assert c["thresholds"][0.5]["both"] == 5


def test_event_log(tmp_path):
    log = EventLog(str(tmp_path / "ev.jsonl"))
    with log.span("trial", name="x"):
        log.emit("epoch", loss=1.0)
    ev = read_events(tmp_path / "ev.jsonl")
    assert [e["event"] for e in ev] == ["trial_start", "epoch", "trial_end"]
    assert ev[-1]["seconds"] >= 0 and json.dumps(ev)


def test_graph_export(tmp_path):
    from featurenet_amd.ir.compile import compile_model
    from featurenet_amd.ir.parse import parse_feature_model
    from featurenet_amd.utils.graph import export, summary

    net = compile_model(parse_feature_model("keras", name="k"), (32, 32, 3), 10)
    p = export(net, tmp_path / "k")
    g = json.loads(open(p["json"]).read())
    assert len(g["nodes"]) == len(net.prog) and g["params"] == net.nb_params
    assert open(p["dot"]).read().startswith("digraph")
    assert "params:" in summary(net)


def _synthetic_report(path, n=20, epochs=12):
    lines = []
    for i in range(n):
        h = "acc#" + "#".join(f"{0.1 + 0.03 * e:.3f}" for e in range(epochs)) + \
            "|val_acc#" + "#".join(f"{0.1 + 0.02 * e + 0.001 * i:.3f}" for e in range(epochs))
        lines.append(f"\r\n{i}: {0.3 + 0.01 * i:.3f} False {10 + i} {1000 * (i + 1)} 0 {h}")
    path.write_text("".join(lines))
    return path


def test_efficiency_overfitting_and_comparison_plots(tmp_path):
    rep = _synthetic_report(tmp_path / "report.txt")
    assert analysis.training_time(rep) == {"n": 20, "sum": float(sum(range(10, 30))), "median": 19.5, "mean": 19.5}
    for fn, name in ((analysis.efficiency, "eff.svg"), (analysis.compare_accuracy, "cmp.svg"),
                     (analysis.overfitting, "over.svg")):
        svg = fn(rep, tmp_path / name).read_text()
        assert svg.startswith("<svg") and svg.rstrip().endswith("</svg>")
    over = (tmp_path / "over.svg").read_text()
    assert over.count("<g transform") == 20 and "architecture 19 49.00% 0.02M" in over
    assert (tmp_path / "cmp.svg").read_text().count("<polyline") == 4      # 2 groups x (train, test)


def test_feature_attribution_on_reference_products(tmp_path):
    import pytest
    from pathlib import Path

    pdt = Path("/root/reference/datasets/10Products.pdt")
    if not pdt.exists():
        pytest.skip("reference product file not available")
    rep = _synthetic_report(tmp_path / "report.txt", n=10)
    res = analysis.feature_attribution(rep, pdt)
    assert len(res["accuracy"]) == 10 and len(res["n_features_per_product"]) == 10
    assert res["n_features_per_product"][0] == 1448                           # SURVEY 2.3 #30a
    # a feature enabled in every product averages all ten accuracies
    full = [v for v in res["features"].values() if v["n"] == 10]
    assert full and all(abs(v["avg"] - np.mean(res["accuracy"])) < 1e-9 for v in full)
    assert res["lowest"][0][1]["avg"] <= res["highest"][0][1]["avg"]
    paths = analysis.plot_feature_attribution(rep, pdt, tmp_path / "feat")
    assert len(paths) == 4 and all(p.exists() for p in paths)
