"""Where a NAS candidate's trial time goes on the GPU (round-4 verdict: "break down the ~0.5 s
per-candidate fixed cost"): dataset load, IR compile + module build, Trainer init (flat
parameters, buckets), the first steps before the graph exists (eager warm-up + capture),
graph replays, per-epoch validation, PreciseBN recalibration, the final evaluation, robustness.

Boundaries are synchronised; graph replays are not (they are timed as the remainder of fit).

    python scripts/r4/trial_phases.py [--candidates 8] [--epochs 5] [--attacks cw,pgd]
"""
import argparse
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from featurenet_amd.ir import compile as IC  # noqa: E402
from featurenet_amd.ir.parse import parse_feature_model  # noqa: E402
from featurenet_amd.robust import evaluate as RE  # noqa: E402
from featurenet_amd.search import trial as T  # noqa: E402
from featurenet_amd.search.mutation import MutationConfig, Mutator  # noqa: E402
from featurenet_amd.training import data as D  # noqa: E402
from featurenet_amd.training import trainer as TR  # noqa: E402

acc = collections.defaultdict(float)
cnt = collections.Counter()


def timed(obj, name, key, pred=None):
    f = getattr(obj, name)

    def g(*a, **k):
        if pred is not None and not pred(*a, **k):
            cnt[key + " (async)"] += 1
            return f(*a, **k)
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = f(*a, **k)
        torch.cuda.synchronize()
        acc[key] += time.perf_counter() - t
        cnt[key] += 1
        return r
    setattr(obj, name, g)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--candidates", type=int, default=8)
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--attacks", default="")
    a = ap.parse_args()
    timed(D, "load_dataset", "dataset")
    timed(IC, "compile_model", "compile_model")
    timed(TR.Trainer, "__init__", "trainer_init")
    timed(TR.Trainer, "fit", "fit (total)")
    # steps before a graph exists: eager warm-up steps and the capture (+ its first replay)
    timed(TR.Trainer, "train_step", "steps before the graph (warm-up + capture)",
          pred=lambda self, *a, **k: getattr(self, "_graph", None) is None)
    timed(TR.Trainer, "evaluate", "evaluate (val + final)")
    timed(TR.Trainer, "recalibrate_bn", "recalibrate_bn")
    timed(RE, "eval_robustness", "eval_robustness")      # (run_trial imports it at call time)
    mut = Mutator(MutationConfig(seed=0))
    base = parse_feature_model("lenet5", name="lenet5")
    specs = [base] + [mut.generate_mutant(base, 0.1) for _ in range(a.candidates - 1)]
    for i, s in enumerate(specs):
        s.name = f"c{i}"
    cfg = T.TrialConfig(dataset="cifar", epochs=a.epochs, batch_size=64, synthetic_sizes=(6000, 1000), graph=True,
                        attacks=[x for x in a.attacks.split(",") if x])
    T.run_trial(specs[0], cfg, device="cuda")              # process warm-up (kernel module, allocator)
    acc.clear()
    cnt.clear()
    t0 = time.perf_counter()
    out = [T.run_trial(s, cfg, device="cuda") for s in specs]
    tot = time.perf_counter() - t0
    n = len(specs)
    print(f"{n} trials {tot:.2f} s ({tot / n:.3f} s each); statuses {collections.Counter(s.status for s in out)}")
    fit = acc.get("fit (total)", 0.0)
    inner = sum(v for k, v in acc.items() if k in ("steps before the graph (warm-up + capture)", "evaluate (val + final)",
                                                   "recalibrate_bn"))
    acc["graph replays (fit remainder)"] = max(fit - inner, 0.0)
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
        print(f"{k:45s} {v:7.3f} s  {v / n * 1e3:8.1f} ms/candidate  {cnt.get(k, 0):6d} calls")


if __name__ == "__main__":
    main()
