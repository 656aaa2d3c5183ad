"""conv_tile plan sweep with the simulated ds_read_b128 bank ways of every plan: the forward (with
BN statistics) and dgrad of the FeatureNet-3D convs (batch 128) under the 1st..6th cheapest plans
of the cost model (FN_TILE_PLAN_RANK), so the bank-conflict term of the planner can be checked
against time."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from featurenet_amd.ops import conv_tile as ct  # noqa: E402
from featurenet_amd.ops.spec import ConvSpec  # noqa: E402

# (name, input size, Cin, Cout, k): the stem runs on its space-to-depth input (32^3 x 8, 4^3 taps)
LAYERS = [("stem", 32, 8, 32, 4), ("conv2", 29, 32, 32, 5), ("conv3", 25, 32, 64, 4), ("conv4", 22, 64, 64, 3)]
RANKS = int(os.environ.get("SWEEP_RANKS", "5"))


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def plan_at(kind, spec, r):
    os.environ["FN_TILE_PLAN_RANK"] = str(r)
    ct._PLANS.clear()
    return ct.fwd_plan(spec) if kind == "fwd" else ct.dgrad_plan(spec)


for name, S, C, K, k in LAYERS:
    x = torch.randn(128, S, S, S, C, device="cuda").to(torch.bfloat16)
    spec = ConvSpec.make(x.shape, K, k, 1, "valid")
    w = torch.randn(K, k, k, k, C, device="cuda") * 0.05
    dy = torch.randn(spec.out_shape5, device="cuda").to(torch.bfloat16)
    kd = (k, k, k)
    for kind in ("fwd", "dgrad") if name != "stem" else ("fwd",):
        # two passes over the plans (the second in reverse order): the first timing of a layer
        # runs on a ramping clock
        for r in list(range(RANKS)) + list(range(RANKS - 1, -1, -1)):
            p = plan_at(kind, spec, r)
            if p is None:
                continue
            if kind == "fwd":
                geom = ct.geometry(p, tuple(x.shape), (spec.OD, spec.OH, spec.OW), kd, (0, 0, 0))
                wpk = ct.pack_weights(w, spec.K, spec.taps, spec.C, p, dgrad=False)
                y = torch.empty(spec.out_shape5, dtype=torch.bfloat16, device="cuda")
                st = torch.empty(ct.workers(p, geom, K), 2, K, dtype=torch.float32, device="cuda")
                fn = lambda: ct.run(x, wpk, None, y, st, p, geom, kd, K, 0)   # noqa: E731
            else:
                geom = ct.geometry(p, (spec.N, spec.OD, spec.OH, spec.OW, spec.K), (spec.D, spec.H, spec.W), kd,
                                   (k - 1, k - 1, k - 1))
                wpk = ct.pack_weights(w, spec.K, spec.taps, spec.C, p, dgrad=True)
                y = torch.empty(x.shape, dtype=torch.bfloat16, device="cuda")
                fn = lambda: ct.run(dy, wpk, None, y, None, p, geom, kd, C, 0)   # noqa: E731
            t = timeit(fn)
            print(json.dumps({"layer": name, "kind": kind, "rank": r, "tile": [p.TD, p.TH, p.TW], "CS": p.CS,
                              "MT": p.MT, "model_cost": round(p.cost), "bank_ways": round(ct.bank_ways(p, kd), 3),
                              "us": round(t, 1)}), flush=True)
os.environ["FN_TILE_PLAN_RANK"] = "0"
