"""Per-shape census of the NAS candidates' convolution calls (eager steps): every call of the
conv entry points of ops/conv.py timed with a device sync around it, grouped by (entry, layer
shape).  Which LeNet-mutant shapes the gather (igemm) kernels still take, and what they cost."""
import collections
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import importlib  # noqa: E402

C = importlib.import_module("featurenet_amd.ops.conv")   # (ops.conv is also a function name)

STATS = collections.defaultdict(lambda: [0, 0.0])


def _key(name, spec):
    return (name, spec.N, (spec.D, spec.H, spec.W), spec.C, spec.K, (spec.KD, spec.KH, spec.KW),
            (spec.sd, spec.sh, spec.sw), (spec.pd, spec.ph, spec.pw))


def wrap(name, spec_arg):
    f = getattr(C, name)

    def g(*a, **k):
        spec = a[spec_arg] if len(a) > spec_arg else k.get("spec")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = f(*a, **k)
        torch.cuda.synchronize()
        s = STATS[_key(name, spec)]
        s[0] += 1
        s[1] += time.perf_counter() - t0
        return r
    setattr(C, name, g)


wrap("native_conv_fwd", 4)
wrap("native_conv_dgrad", 2)
wrap("native_conv_wgrad", 2)
wrap("igemm_wgrad_cropped", 2)

from featurenet_amd.ir.parse import parse_feature_model  # noqa: E402
from featurenet_amd.search.mutation import MutationConfig, Mutator  # noqa: E402
from featurenet_amd.search.trial import TrialConfig, TrialScheduler  # noqa: E402

mut = Mutator(MutationConfig(seed=0))
base = parse_feature_model("lenet5", name="lenet5")
specs = [base] + [mut.generate_mutant(base, 0.1) for _ in range(int(os.environ.get("NCAND", "8")) - 1)]
for i, s in enumerate(specs):
    s.name = f"c{i}"
sched = TrialScheduler(mode="inline", workers_per_device=1)
cfg = TrialConfig(dataset="cifar", epochs=1, batch_size=64, synthetic_sizes=(6000, 1000), graph=False)
out = sched.map(specs, cfg)
tot = sum(v[1] for v in STATS.values())
print(json.dumps({"trained": sum(s.status == "trained" for s in out), "conv_call_seconds": round(tot, 3)}))
print("| entry | N | in DHW | C | K | taps | stride | pad | calls | ms | % |")
print("|---|---|---|---|---|---|---|---|---|---|---|")
for k, (n, t) in sorted(STATS.items(), key=lambda kv: -kv[1][1])[:40]:
    print("| " + " | ".join(str(x) for x in k) + f" | {n} | {t * 1e3:.1f} | {100 * t / tot:.1f} |")
