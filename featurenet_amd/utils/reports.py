"""Result records and log formats shared with the reference tooling.

Reference formats kept bit-compatible so the reference's plotters / UI can
read our sessions:

* ``KerasFeatureVector`` (``model/keras_model.py:23-56``): the genome/result
  record ``[accuracy, [name, [nb_blocks, nb_layers, nb_params, nb_flops],
  [robustness_score, [clever, fgsm, pgd, cw]], metrics], *feature_bits]``,
  with bit-flip mutation (rate 0.05) and one-point crossover;
* population log lines ``"\\r\\n{idx} {unix_ts}:{json(vector)}"`` in
  ``e{n}.json`` / ``base.json`` (``full_evolution.py:131,155,263``);
* batch-trainer report lines ``"\\r\\n{idx}: {acc} {stop} {time} {params} {flops} {hist}"``
  (``full.py:16``) consumed by ``plots/plotter.py:6-17`` and ``correlation.py:5-16``.
"""
from __future__ import annotations

import json
import random
import re
import time
from pathlib import Path


class KerasFeatureVector:
    def __init__(self, accuracy, attributes, features):
        self.accuracy = accuracy
        self.attributes = attributes
        self.features = list(features)

    def mutate(self, rate: float = 0.05, rng: random.Random | None = None) -> None:
        r = rng or random
        self.features = [f if r.random() > rate else 1 - f for f in self.features]

    def cross_over(self, other: "KerasFeatureVector", crossover_type: str = "onepoint",
                   rng: random.Random | None = None) -> "KerasFeatureVector":
        r = rng or random
        point = r.randint(0, len(self.features))
        return KerasFeatureVector(0, [0, 0, 0, 0], self.features[:point] + other.features[point:])

    def to_vector(self) -> list:
        return [self.accuracy] + [self.attributes] + self.features

    @staticmethod
    def from_vector(v: list) -> "KerasFeatureVector":
        return KerasFeatureVector(v[0], v[1], v[2:])

    @property
    def fitness(self) -> float:
        return 0 if self.accuracy is None else self.accuracy

    @property
    def name(self) -> str:
        try:
            return self.attributes[0]
        except Exception:
            return ""

    @property
    def robustness_score(self) -> float:
        try:
            return float(self.attributes[2][0])
        except Exception:
            return 0.0

    def __str__(self) -> str:
        return "{}:{}".format(";".join(str(i) for i in self.attributes), self.accuracy)


def _score0(v):
    if isinstance(v, (list, tuple)):
        return v[0] if v else 0
    return v or 0


def spec_vector(spec) -> KerasFeatureVector:
    """ModelSpec -> KerasFeatureVector (``KerasFeatureModel.to_kerasvector``)."""
    attrs = [spec.name, [len(spec.blocks), spec.nb_layers, spec.nb_params, spec.nb_flops],
             [spec.robustness_score, [spec.clever_score, spec.fgsm_score, spec.pgd_score, spec.cw_score]],
             spec.metrics]
    return KerasFeatureVector(spec.accuracy, attrs, list(spec.features))


def population_line(index: int, vector: list, ts: int | None = None) -> str:
    return "\r\n{} {}:{}".format(index, int(time.time()) if ts is None else ts, json.dumps(vector))


def append_population(path: str | Path, population, start_index: int = 0) -> None:
    with open(path, "a") as f:
        for i, spec in enumerate(population):
            f.write(population_line(start_index + i, spec_vector(spec).to_vector()))


_POP_LINE = re.compile(r"^(\d+) (\d+):(.*)$")


def read_population(path: str | Path) -> list[tuple[int, int, list]]:
    out = []
    for line in Path(path).read_text().splitlines():
        m = _POP_LINE.match(line.strip())
        if m:
            out.append((int(m.group(1)), int(m.group(2)), json.loads(m.group(3))))
    return out


def report_line(index: int, accuracy: float, stop_training: bool, train_time: float, params: int, flops: int,
                history: dict) -> str:
    hist = "|".join(f"{k}#{'#'.join(str(round(v, 5)) for v in vals)}" for k, vals in history.items()
                    if isinstance(vals, list))
    return f"\r\n{index}: {accuracy} {stop_training} {train_time} {params} {flops} {hist}"


_REPORT = re.compile(r"^(\d+): (\S+) (\S+) (\S+) (\S+) (\S+) ?(.*)$")


def read_report(path: str | Path) -> list[dict]:
    rows = []
    for line in Path(path).read_text().splitlines():
        m = _REPORT.match(line.strip())
        if not m:
            continue
        hist = {}
        for part in (m.group(7) or "").split("|"):
            if "#" in part:
                k, *vals = part.split("#")
                hist[k] = [float(v) for v in vals if v]
        rows.append({"index": int(m.group(1)), "accuracy": float(m.group(2)), "stop": m.group(3) == "True",
                     "time": float(m.group(4)), "params": int(float(m.group(5))), "flops": int(float(m.group(6))),
                     "history": hist})
    return rows
