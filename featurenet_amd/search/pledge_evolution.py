"""Diversity-driven NAS through feature-model constraints (reference
``PledgeEvolution``, ``pledge_evolution.py:53-270``).

* ``end2end``: expand the 1-block / 1-cell template FM to B x C
  (:func:`featurenet_amd.fm.extend.generate_featuretree`);
* ``run``: sample N diverse products (native PLEDGE-equivalent sampler), train
  them all, then per generation keep the top ``ceil(5% N)`` by accuracy; for
  each survivor and each of two batches write a child FM that forbids a random
  subset (ratio ``0.2 + 0.75*evo/E``) of the survivor's enabled leaf features
  (constraints ``~Architecture or ~<label>``), sample ``max(3, ceil(0.5 *
  per_parent))`` products from it, train and merge;
* resume from the ``{N}products[_e{n}].json`` vector lists.

Population records are :class:`KerasFeatureVector` lists exactly as the
reference writes them, and full IR specs are kept alongside.
"""
from __future__ import annotations

import json
import math
import os
import random
import re
import xml.etree.ElementTree as ET
from dataclasses import dataclass
from pathlib import Path

from ..fm.extend import generate_featuretree
from ..fm.products import ProductSet
from ..fm.sampler import default_pledge_output, run_pledge
from ..ir.parse import parse_feature_model
from ..utils.reports import KerasFeatureVector, spec_vector
from .trial import TrialConfig, TrialScheduler


@dataclass
class PledgeResult:
    session_path: str
    population: list        # KerasFeatureVector
    specs: list


def end2end(base_path: str | Path, nb: tuple, input_file: str | Path, block_features: bool = False) -> str:
    nb_blocks, nb_cells, nb_products = (int(v) for v in nb)
    Path(base_path).mkdir(parents=True, exist_ok=True)
    full = f"{base_path}/nas_{nb_blocks}_{nb_cells}_{nb_products}.xml"
    if not os.path.isfile(full):
        generate_featuretree(input_file, full, nb_cells, nb_blocks, block_features=block_features)
    return full


def extract_leaves(pdt_path: str | Path):
    ps = ProductSet(pdt_path, binary_products=True)
    return ps, {"filtered_features_label": ProductSet.filter_leaves(ps.features), "products": []}


def generate_children(mutant_path: str, mutant_labels: list, initial_fm: str, nb_products: int,
                      constraints_ratio: float, rng: random.Random, duration_s: float = 2.0, seed: int = 0) -> str:
    labels = [m for m in mutant_labels if rng.random() < constraints_ratio]
    tree = ET.parse(initial_fm)
    cons = list(tree.getroot())[1]
    raw = (cons.text or "").split("\n")
    n = len(raw)
    raw = raw[:-1]
    for i, lbl in enumerate(labels):
        raw.append(f"C{n + i - 1}:~Architecture  or  ~{lbl}")
    cons.text = "\n".join(raw)
    dst = f"{mutant_path}.xml"
    tree.write(dst, encoding="UTF-8", xml_declaration=True)
    out = f"{dst[:-4]}.pdt"
    run_pledge(dst, int(nb_products), out, duration=duration_s, seed=seed)
    return out


def train_products(product_set: ProductSet, scheduler: TrialScheduler, cfg: TrialConfig, max_products: int = 0,
                   prefix: str = "p") -> list:
    specs = []
    for i, (tree, feats) in enumerate(product_set.format_products()):
        bits = feats if product_set.binary_products else sorted(feats, key=lambda k: abs(int(k)))
        s = parse_feature_model(tree, name=f"{prefix}{i:04d}")
        s.features = [1 if int(v) > 0 else 0 for v in bits]
        specs.append(s)
        if max_products and i + 1 >= max_products:
            break
    return scheduler.map(specs, cfg)


def run(base_path: str, input_file: str, output_file: str = "", last_pdts_path: str = "",
        nb_base_products: int = 100, dataset: str = "cifar", training_epochs: int = 25, evolution_epochs: int = 50,
        attacks=("cw",), scheduler: TrialScheduler | None = None, trial: TrialConfig | None = None,
        pledge_duration_s: float = 10.0, seed: int = 0, verbose: int = 1) -> PledgeResult:
    rng = random.Random(seed)
    Path(base_path).mkdir(parents=True, exist_ok=True)
    sp = Path(base_path) / dataset
    sp.mkdir(parents=True, exist_ok=True)
    survival_count = math.ceil(0.05 * nb_base_products)
    per_parent = int((nb_base_products - survival_count) / survival_count)
    scheduler = scheduler or TrialScheduler()
    cfg = trial or TrialConfig(dataset=dataset, epochs=training_epochs)
    cfg.dataset, cfg.epochs, cfg.attacks = dataset, training_epochs, list(attacks)
    output_file = output_file or default_pledge_output(base_path, nb_base_products)
    last_pdts_path = last_pdts_path or str(sp / f"{nb_base_products}products.json")

    def log(msg):
        if verbose:
            print(f"[pledge-evolution] {msg}", flush=True)

    if not os.path.isfile(output_file):
        log(f"initial sampling of {nb_base_products} products from {input_file}")
        run_pledge(input_file, nb_base_products, output_file, duration=pledge_duration_s, seed=seed)
    product_set, pop = extract_leaves(output_file)
    specs: list = []
    last_epoch = 0
    if os.path.isfile(last_pdts_path):
        pop["products"] = [KerasFeatureVector.from_vector(v) for v in json.loads(Path(last_pdts_path).read_text())]
        m = re.findall(r"products_e(\d+)\.json", last_pdts_path)
        if m:
            last_epoch = int(m[0]) + 1
        log(f"resumed {len(pop['products'])} trained products from {last_pdts_path}")
    else:
        specs = train_products(product_set, scheduler, cfg, nb_base_products, prefix="initial_")
        pop["products"] = [spec_vector(s) for s in specs]
        Path(last_pdts_path).write_text(json.dumps([v.to_vector() for v in pop["products"]]))
    labels = pop["filtered_features_label"]
    for evo in range(evolution_epochs):
        ratio = 0.2 + 0.75 * evo / max(evolution_epochs, 1)
        batches = [(ratio, 0.5), (ratio, 0.5)]
        survivors = sorted(pop["products"], key=lambda v: v.accuracy or 0, reverse=True)[:survival_count]
        surv_labels = [[labels[k] for k in labels if int(k) - 1 < len(s.features) and s.features[int(k) - 1] == 1]
                       for s in survivors]
        pop["products"] = survivors
        for i in range(len(survivors)):
            for b, (r, nb) in enumerate(batches):
                mid = f"e{evo}_m{i}_b{b}"
                mpath = str(sp / mid)
                pdt = generate_children(mpath, surv_labels[i], input_file, max(3, math.ceil(nb * per_parent)), r, rng,
                                        duration_s=pledge_duration_s, seed=seed + evo * 1000 + i * 10 + b)
                try:
                    ps = ProductSet(pdt, binary_products=True)
                except Exception as e:
                    log(f"skipping {pdt}: {e}")
                    continue
                child_specs = train_products(ps, scheduler, cfg, prefix=f"{mid}_")
                specs += child_specs
                vecs = sorted((spec_vector(s) for s in child_specs), key=lambda v: v.accuracy or 0, reverse=True)
                Path(f"{mpath}.json").write_text(json.dumps([v.to_vector() for v in vecs]))
                pop["products"] += vecs
        ranked = sorted(pop["products"], key=lambda v: v.accuracy or 0, reverse=True)
        Path(sp / f"{nb_base_products}products_e{evo + last_epoch}.json").write_text(
            json.dumps([v.to_vector() for v in ranked]))
        log(f"generation {evo + last_epoch}: {len(ranked)} products, top accuracy "
            f"{ranked[0].accuracy if ranked else 0:.4f}")
    return PledgeResult(str(sp), pop["products"], specs)
