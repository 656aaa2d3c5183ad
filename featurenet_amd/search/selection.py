"""Survivor selection (reference ``FullEvolution.get_fronts`` / ``select``,
``full_evolution.py:40-105``; strategies from ``mutable_base.py:9-11``).

* ELITIST: keep the ``survival_count`` best (population sorted by accuracy).
* HYBRID (reference default): ``ceil(sc/4)`` elites + the rest drawn with
  replacement from softmax(accuracy).
* PARETO: restrict to the first non-dominated front of (accuracy, robustness)
  when it has more than one member, score = acc/max * rob/max, sort ascending
  (as the reference does), then HYBRID-style elites + softmax draws.
"""
from __future__ import annotations

import math

import numpy as np

from .mutation import SelectionStrategies


def get_fronts(accuracy, robustness) -> list[int]:
    """Indices of the first non-dominated front (strict dominance on both objectives)."""
    n = len(accuracy)
    front = []
    for i in range(n):
        dominated = False
        for j in range(n):
            if i != j and accuracy[j] > accuracy[i] and robustness[j] > robustness[i]:
                dominated = True
                break
        if not dominated:
            front.append(i)
    return front


def select(population: list, survival_count: int, strategy=SelectionStrategies.HYBRID,
           rng: np.random.Generator | None = None) -> list:
    rng = rng or np.random.default_rng()
    pop = list(population)
    if not pop:
        return []
    x = np.array([float(p.accuracy) for p in pop])
    score = x
    if strategy == SelectionStrategies.PARETO and len(pop) > 1:
        y = np.array([float(p.robustness_score) for p in pop])
        front = get_fronts(x, y)
        if len(front) > 1:
            pop = [pop[i] for i in front]
            xf, yf = x[front], y[front]
            mx, my = (xf.max() or 1.0), (yf.max() or 1.0)
            score = xf / mx * yf / my
            order = np.argsort(score, kind="stable")       # ascending, as the reference
            pop = [pop[i] for i in order]
            score = score[order]
    e = np.exp(score - np.max(score))
    prob = e / e.sum()
    elitist = survival_count if strategy == SelectionStrategies.ELITIST else math.ceil(survival_count / 4)
    fittest = pop[:min(len(pop), elitist)]
    for _ in range(min(len(pop), survival_count - elitist)):
        fittest.append(pop[int(rng.choice(len(pop), p=prob))])
    return fittest
