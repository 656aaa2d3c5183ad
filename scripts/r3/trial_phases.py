"""Where a NAS candidate's trial time goes (GPU): dataset, build, Trainer init, train steps
(eager warm-up + graph capture + replays), validation, precise-BN recalibration, final eval."""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from featurenet_amd.ir.parse import parse_feature_model  # noqa: E402
from featurenet_amd.search.mutation import MutationConfig, Mutator  # noqa: E402
from featurenet_amd.search import trial as T  # noqa: E402
from featurenet_amd.training import trainer as TR  # noqa: E402
from featurenet_amd.ir import compile as IC  # noqa: E402
from featurenet_amd.training import data as D  # noqa: E402

acc = collections.defaultdict(float)
cnt = collections.Counter()


def wrap(obj, name, key):
    f = getattr(obj, name)

    def g(*a, **k):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = f(*a, **k)
        torch.cuda.synchronize()
        acc[key] += time.perf_counter() - t
        cnt[key] += 1
        return r
    setattr(obj, name, g)


wrap(TR.Trainer, "train_step", "train_step")
wrap(TR.Trainer, "evaluate", "evaluate")
wrap(TR.Trainer, "recalibrate_bn", "recalibrate_bn")
wrap(TR.Trainer, "__init__", "trainer_init")
wrap(T, "load_dataset", "load_dataset") if hasattr(T, "load_dataset") else None
wrap(D, "load_dataset", "load_dataset")
wrap(IC, "compile_model", "compile_model")
mut = Mutator(MutationConfig(seed=0))
base = parse_feature_model("lenet5", name="lenet5")
specs = [base] + [mut.generate_mutant(base, 0.1) for _ in range(7)]
cfg = T.TrialConfig(dataset="cifar", epochs=5, batch_size=64, synthetic_sizes=(6000, 1000), graph=True)
T.run_trial(specs[0], cfg, device="cuda")
acc.clear(); cnt.clear()
t0 = time.perf_counter()
for s in specs:
    T.run_trial(s, cfg, device="cuda")
tot = time.perf_counter() - t0
print(f"{len(specs)} trials {tot:.2f} s ({tot / len(specs):.3f} s each)")
for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
    print(f"{k:16s} {v:7.3f} s  {cnt[k]:6d} calls  {v / max(cnt[k], 1) * 1e3:8.2f} ms/call")
