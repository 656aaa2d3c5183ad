"""Mutation-driven NAS over accuracy x robustness (reference ``FullEvolution``,
``full_evolution.py:35-276``).

Session layout (reference-compatible): ``{base}/{dataset}/ee{E}_te{T}_mr{m}_sr{s}[_{ts}]/``
with ``base.json`` (initial population), ``e{n}.json`` (each generation, one
``"\\r\\n{idx} {ts}:{vector}"`` line per model) and a per-generation snapshot
``{N}products_e{n}.json`` (the reference writes an empty pickle here, so its
resume never worked; ours is an atomic JSON list of full IR specs + results,
and ``resume_from`` picks it up).

Per generation: ``select`` survivors -> ``evolve`` (each survivor breeds with a
random survivor and is mutated ``Binomial(100, mutation_rate)`` times under
CHOICE) -> train every untrained candidate (concurrently through the
:class:`~featurenet_amd.search.trial.TrialScheduler`, one per GPU) ->
robustness for accurate ones -> log -> keep accuracy > 0.1, sorted.
Initial population: a resume snapshot, else a PLEDGE product file
(``products_{T}s_{B}_{C}_{N}.pdt`` or any ``.pdt``), else a template
(``lenet5`` by default) trained first.
"""
from __future__ import annotations

import json
import math
import os
import re
import time
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np

from ..fm.products import ProductSet
from ..ir.parse import parse_feature_model
from ..ir.spec import ModelSpec
from ..utils.reports import append_population
from .mutation import MutationConfig, MutationStrategies, Mutator, SelectionStrategies
from .selection import select
from .trial import TrialConfig, TrialScheduler


@dataclass
class EvolutionResult:
    session_path: str
    population: list
    generations: int
    history: list = field(default_factory=list)


def session_dir(base_path: str, dataset: str, evolution_epochs: int, training_epochs: int, mutation_rate: float,
                survival_rate: float) -> Path:
    base = Path(base_path) / dataset
    base.mkdir(parents=True, exist_ok=True)
    s = base / f"ee{evolution_epochs}_te{training_epochs}_mr{mutation_rate}_sr{survival_rate}"
    if s.exists():
        s = Path(f"{s}_{int(time.time())}")
    s.mkdir(parents=True)
    return s


def save_snapshot(path: Path, population: list) -> None:
    tmp = path.with_suffix(".tmp")
    tmp.write_text(json.dumps([p.to_dict() for p in population]))
    tmp.replace(path)


def load_snapshot(path: str | Path) -> list:
    return [ModelSpec.from_dict(d) for d in json.loads(Path(path).read_text())]


def specs_from_products(pdt_path: str | Path) -> list:
    ps = ProductSet(pdt_path)
    specs = []
    for i, (tree, feats) in enumerate(ps.format_products()):
        s = parse_feature_model(tree, name=f"p{i:04d}", product_features=sorted(feats, key=lambda k: abs(int(k))))
        specs.append(s)
    return specs


def evolve(parents: list, nb_product_perparent: int, mutator: Mutator, mutation_ratio: float, breed: bool = True,
           generation: int = 0) -> list:
    children = []
    for i, p in enumerate(parents):
        for j in range(nb_product_perparent):
            base = mutator.breed(p, parents[int(mutator.rng.integers(len(parents)))]) if breed else p.clone()
            child = mutator.generate_mutant(base, mutation_ratio)
            child.name = f"e{generation}_{i}_{j}"
            child.features = list(p.features)
            children.append(child)
    return list(parents) + children


def run_evolution(base_path: str = "runs", last_pdts_path: str = "", nb_base_products: int = 100,
                  dataset: str = "cifar", training_epochs: int = 25, mutation_rate: float = 0.1,
                  survival_rate: float = 0.1, breed: bool = True, evolution_epochs: int = 50, model: str = "",
                  attacks=("cw", "pgd"), mutation_strategy: MutationStrategies = MutationStrategies.CHOICE,
                  selection_strategy: SelectionStrategies = SelectionStrategies.HYBRID, max_nb_cells: int = 10,
                  max_nb_blocks: int = 20, resume_from: str = "", scheduler: TrialScheduler | None = None,
                  trial: TrialConfig | None = None, seed: int = 0, verbose: int = 1) -> EvolutionResult:
    sp = session_dir(base_path, dataset, evolution_epochs, training_epochs, mutation_rate, survival_rate)
    survival_count = max(3, math.ceil(survival_rate * nb_base_products))
    per_parent = math.ceil((nb_base_products - survival_count) / survival_count)
    mutator = Mutator(MutationConfig(mutation_strategy, selection_strategy, max_nb_cells, max_nb_blocks, seed))
    rng = np.random.default_rng(seed)
    scheduler = scheduler or TrialScheduler()
    tcfg = trial or TrialConfig(dataset=dataset, epochs=training_epochs)
    tcfg.dataset, tcfg.epochs = dataset, training_epochs
    tcfg.attacks = list(attacks)
    tcfg.save_dir = tcfg.save_dir or str(sp / "models")

    def log(msg):
        if verbose:
            print(f"[evolution] {msg}", flush=True)

    start_epoch = 0
    resume = resume_from or (last_pdts_path if re.search(r"products_e(\d+)\.json$", last_pdts_path or "") else "")
    if resume and os.path.isfile(resume):
        population = load_snapshot(resume)
        m = re.search(r"_e(\d+)\.json$", resume)
        start_epoch = int(m.group(1)) if m else 0     # next generation is start_epoch + 1
        log(f"resuming {len(population)} individuals from {resume} at generation {start_epoch}")
    elif last_pdts_path and os.path.isfile(last_pdts_path):
        initial = specs_from_products(last_pdts_path)
        log(f"training {len(initial)} PLEDGE products from {last_pdts_path}")
        tcfg.save_prefix = "base_"
        population = scheduler.map(initial, tcfg)
        append_population(sp / "base.json", population)
    else:
        name = model or "lenet5"
        seed_spec = parse_feature_model(name, name=name)
        tcfg.save_prefix = "base_"
        population = scheduler.map([seed_spec], tcfg)
        append_population(sp / "e0.json", population)
    population = sorted([p for p in population if p.status != "invalid"], key=lambda p: p.accuracy, reverse=True)
    history = []
    for e in range(start_epoch, start_epoch + evolution_epochs):
        evo = e + 1
        if not population:
            log("population is empty, stopping")
            break
        parents = select(population, survival_count, selection_strategy, rng)
        candidates = evolve(parents, per_parent, mutator, mutation_rate, breed, evo)
        todo = [c for c in candidates if c.status != "trained"]
        tcfg.save_prefix = f"e{evo}_"
        t0 = time.perf_counter()
        trained = {id(c): r for c, r in zip(todo, scheduler.map(todo, tcfg))}
        dt = time.perf_counter() - t0
        candidates = [trained.get(id(c), c) for c in candidates]
        append_population(sp / f"e{evo}.json", candidates)
        population = sorted([c for c in candidates if c.accuracy > 0.1], key=lambda c: c.accuracy, reverse=True)
        save_snapshot(sp / f"{nb_base_products}products_e{evo}.json", population)
        top = population[0].accuracy if population else 0.0
        history.append({"generation": evo, "size": len(population), "top_accuracy": top,
                        "invalid": sum(c.status == "invalid" for c in candidates),
                        "trained": len(todo), "seconds": round(dt, 2)})   # (the generation's trial wall time)
        log(f"generation {evo}: {len(population)} individuals, top accuracy {top:.4f}")
    return EvolutionResult(str(sp), population, len(history), history)
