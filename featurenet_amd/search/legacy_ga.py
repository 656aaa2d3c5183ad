"""Legacy genetic algorithm directly on product bit vectors (reference
``evolution.py:19-129``): truncation selection (survival 0.5), one-point
crossover and bit-flip mutation (rate 0.05) of :class:`KerasFeatureVector`
genomes; individuals without accuracy are (re)trained; one JSON line per
generation.  The reference crashes on its first generation (``.to_vector()``
called on a model, ``evolution.py:69``); this version runs.
"""
from __future__ import annotations

import json
import random
from pathlib import Path

from ..fm.products import ProductSet
from ..ir.parse import parse_feature_model
from ..utils.reports import KerasFeatureVector, spec_vector
from .trial import TrialConfig, TrialScheduler


def _train_vectors(vectors: list, ps: ProductSet, scheduler: TrialScheduler, cfg: TrialConfig) -> list:
    todo, specs = [], []
    for i, v in enumerate(vectors):
        if v.accuracy:
            continue
        tree, _ = ps.format_product(original_product=[1 if b else 0 for b in v.features])
        s = parse_feature_model(tree, name=f"ga{i:04d}")
        s.features = list(v.features)
        specs.append(s)
        todo.append(i)
    for i, s in zip(todo, scheduler.map(specs, cfg)):
        vectors[i] = spec_vector(s)
    return vectors


def run(pdt_path: str, output_path: str, generations: int = 10, survival_rate: float = 0.5,
        mutation_rate: float = 0.05, scheduler: TrialScheduler | None = None, cfg: TrialConfig | None = None,
        seed: int = 0) -> list:
    rng = random.Random(seed)
    ps = ProductSet(pdt_path, binary_products=True)
    scheduler = scheduler or TrialScheduler()
    cfg = cfg or TrialConfig()
    out = Path(output_path)
    pop = []
    if out.exists():   # resume from the last logged generation
        lines = [l for l in out.read_text().splitlines() if l.strip()]
        if lines:
            pop = [KerasFeatureVector.from_vector(v) for v in json.loads(lines[-1])]
    if not pop:
        pop = [KerasFeatureVector(0, [0, 0, 0, 0], list(p)) for p in ps.products]
    pop = _train_vectors(pop, ps, scheduler, cfg)
    n = len(pop)
    for _ in range(generations):
        pop.sort(key=lambda v: v.fitness, reverse=True)
        keep = pop[:max(2, int(n * survival_rate))]
        children = []
        while len(keep) + len(children) < n:
            a, b = rng.sample(keep, 2)
            c = a.cross_over(b, rng=rng)
            c.mutate(mutation_rate, rng=rng)
            children.append(c)
        pop = _train_vectors(keep + children, ps, scheduler, cfg)
        with open(out, "a") as f:
            f.write(json.dumps([v.to_vector() for v in pop]) + "\n")
    return pop
