"""PLEDGE-equivalent product sampling (native C++ ``_rt.sample_diverse``).

Reference: ``run_pledge`` (``pledge_evolution.py:36-47``) shells out to
``java -jar PLEDGE.jar generate_products -fm F -nbProds N -o OUT
-timeAllowedMS T``.  Here the same contract is served in-process by the
native sampler: the FM is parsed (:mod:`.splot`), lowered to CNF, and the
(1+1) diversity EA runs for ``duration_s`` seconds; the ``.pdt`` written uses
the same ``id->label`` header + signed-id product lines PLEDGE emits.
"""
from __future__ import annotations

import time
from pathlib import Path

from .. import _native
from . import splot
from .products import ProductSet


def sample_products(fm: splot.FeatureModel, nb_products: int, duration_s: float = 1.0, seed: int = 0,
                    prioritize: bool = True) -> dict:
    nvars, clauses = fm.to_cnf()
    rt = _native.runtime()
    res = rt.sample_diverse(nvars, clauses, int(nb_products), float(duration_s) * 1000.0, int(seed), 0, prioritize)
    res["labels"] = fm.names()
    return res


def run_pledge(input_file: str | Path, nb_base_products: int, output_file: str | Path, duration: float = 600,
               seed: int = 0) -> int:
    """Drop-in for the reference ``run_pledge``; returns 0 on success (like ``check_call``)."""
    t0 = time.time()
    fm = splot.load(input_file)
    res = sample_products(fm, nb_base_products, duration, seed)
    ProductSet.write(output_file, res["labels"], res["products"])
    res["wall_s"] = time.time() - t0
    return 0


def default_pledge_output(base_path: str | Path, nb_base_products: int) -> str:
    return f"{base_path}/{nb_base_products}products.pdt"
