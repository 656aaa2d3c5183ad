#!/usr/bin/env python3
"""NAS search throughput: candidates trained per hour.

Trains ``--candidates`` mutants of the LeNet-5 template for ``--epochs`` on a
synthetic MNIST- or CIFAR-shaped set (no network) through the TrialScheduler, with and
without hipGraph-captured training steps.  ``--workers-per-device N`` runs N worker
processes per GPU (several small candidates share one MI355X).  The reference's unit of
work is 25 epochs x 100 products (``pledge_evolution.py:20``); ``--candidates 32
--epochs 5`` is the round-3 census workload.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--candidates", type=int, default=8)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--train", type=int, default=6000)
    ap.add_argument("--mode", default="inline", choices=["inline", "process"])
    ap.add_argument("--dataset", default="mnist", choices=["mnist", "cifar"])
    ap.add_argument("--workers-per-device", type=int, default=1)
    ap.add_argument("--graph", default="both", choices=["both", "on", "off"])
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--attacks", default="", help="comma list (e.g. cw,pgd): robustness evaluation of every trained "
                    "candidate with accuracy >= 0.5, as FullEvolution does (full_evolution.py:244-258)")
    ap.add_argument("--robustness-set", type=int, default=500)
    ap.add_argument("--warm", action="store_true",
                    help="start the worker pool (one 1-epoch trial per worker) before the clock: the steady "
                         "state of a multi-generation search, whose workers persist across generations")
    a = ap.parse_args()
    from featurenet_amd.ir.parse import parse_feature_model
    from featurenet_amd.search.mutation import MutationConfig, Mutator
    from featurenet_amd.search.trial import TrialConfig, TrialScheduler

    mut = Mutator(MutationConfig(seed=0))
    base = parse_feature_model("lenet5", name="lenet5")
    specs = [base] + [mut.generate_mutant(base, 0.1) for _ in range(a.candidates - 1)]
    for i, s in enumerate(specs):
        s.name = f"c{i}"
    mode = "process" if a.workers_per_device > 1 else a.mode
    sched = TrialScheduler(mode=mode, workers_per_device=a.workers_per_device)
    graphs = {"both": (False, True), "on": (True,), "off": (False,)}[a.graph]
    for graph in graphs:
        attacks = [t for t in a.attacks.split(",") if t]
        cfg = TrialConfig(dataset=a.dataset, epochs=a.epochs, batch_size=a.batch, synthetic_sizes=(a.train, 1000),
                          graph=graph, attacks=attacks, robustness_set_size=a.robustness_set)
        if a.warm:
            nw = len(sched.slots()) if sched.mode == "process" else 1
            wcfg = TrialConfig(**{**cfg.to_dict(), "epochs": 1, "attacks": []})
            sched.map([s.clone() for s in specs[:nw]], wcfg)
        t0 = time.perf_counter()
        out = sched.map(specs, cfg)
        dt = time.perf_counter() - t0
        ok = sum(s.status == "trained" for s in out)
        print(json.dumps({"metric": "NAS candidates trained per hour", "graph": graph, "value": round(ok / dt * 3600, 1),
                          "warm_workers": bool(a.warm),
                          "candidates": len(specs), "trained": ok, "seconds": round(dt, 2),
                          "devices": sched.devices, "workers_per_device": a.workers_per_device,
                          "dataset": a.dataset, "epochs": a.epochs, "train_samples": a.train, "batch": a.batch,
                          "attacks": attacks, "robustness_set": a.robustness_set if attacks else None,
                          "robustness_evaluated": sum(s.status == "trained" and (s.accuracy or 0) >= 0.5
                                                      for s in out) if attacks else None,
                          # every candidate that did not train, with its status and reason (e.g. c33:
                          # 'invalid', > 20M parameters -- the reference's cap, model/keras_model.py:127)
                          "not_trained": [{"name": s.name, "status": s.status,
                                           "error": (s.error or "").splitlines()[0][:200]}
                                          for s in out if s.status != "trained"]}), flush=True)


if __name__ == "__main__":
    main()
