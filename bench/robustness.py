#!/usr/bin/env python3
"""Robustness-evaluation throughput of one NAS candidate (the CW / PGD / CLEVER
hot loops of ``tensorflow_generator.py:151-218`` and ``model/metrics.py:242-324``).

Trains the LeNet-5 template on the synthetic CIFAR-shaped set for ``--epochs`` (accuracy must
reach the reference's 0.5 gate to be evaluated at all), then runs the reference robustness
policy -- ``--metrics`` on the first ``--set-size`` test samples, CLEVER over ``--clever``
samples (radius 2, 10 batches of 5, pool factor 3) -- and prints one JSON line with the
seconds per metric and per candidate.

    python bench/robustness.py --set-size 500 --clever 500 --metrics clever,pgd,cw
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dataset", default="cifar", choices=["cifar", "mnist"])
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--train", type=int, default=6000)
    ap.add_argument("--set-size", type=int, default=500)
    ap.add_argument("--clever", type=int, default=500)
    ap.add_argument("--metrics", default="clever,pgd,cw")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--census", action="store_true",
                    help="count the native kernel launches of the robustness part by entry point (a counting "
                         "proxy around the _C module): weight-gradient entry points must not appear")
    a = ap.parse_args()
    import torch

    from featurenet_amd.ir.compile import compile_model
    from featurenet_amd.ir.parse import parse_feature_model
    from featurenet_amd.robust.evaluate import eval_robustness
    from featurenet_amd.training.data import load_dataset
    from featurenet_amd.training.trainer import Trainer

    ds = load_dataset(a.dataset, synthetic_sizes=(a.train, max(1000, a.set_size)), seed=0)
    torch.manual_seed(0)
    model = compile_model(parse_feature_model("lenet5", name="lenet5"), ds.input_shape, ds.num_classes)
    tr = Trainer(model, device=a.device, graph=a.device == "cuda")
    t0 = time.time()
    tr.fit(ds.x_train, ds.y_train, epochs=a.epochs, batch_size=64, verbose=0)
    train_s = time.time() - t0
    _, acc = tr.evaluate(ds.x_test, ds.y_test)
    res = {"metric": "robustness evaluation seconds per candidate", "dataset": a.dataset,
           "synthetic": bool(ds.synthetic), "accuracy": round(acc, 4), "train_s": round(train_s, 2),
           "set_size": a.set_size, "clever_samples": a.clever}
    census: dict = {}
    if a.census:
        from featurenet_amd import _native

        real = _native.kernels()

        class Counting:
            def __getattr__(self, name):
                f = getattr(real, name)
                if not callable(f):
                    return f

                def wrap(*args, **kw):
                    census[name] = census.get(name, 0) + 1
                    return f(*args, **kw)
                return wrap

        _native._K = Counting()
    total = 0.0
    for m in [t for t in a.metrics.split(",") if t]:
        if a.device == "cuda":
            torch.cuda.synchronize()
        t1 = time.time()
        r = eval_robustness(tr.model, ds, [m], set_size=a.set_size, clever_samples=a.clever)
        if a.device == "cuda":
            torch.cuda.synchronize()
        dt = time.time() - t1
        total += dt
        res[m + "_s"] = round(dt, 2)
        v = r.get(m)
        res[m] = v if not isinstance(v, tuple) else [round(float(u), 4) for u in v]
        if r.get("errors"):
            res.setdefault("errors", {}).update({k: e.splitlines()[0] for k, e in r["errors"].items()})
    if a.census:
        res["census"] = dict(sorted(census.items(), key=lambda kv: -kv[1]))
        res["wgrad_launches"] = sum(v for k, v in census.items() if "wgrad" in k or "wtile" in k)
    res["value"] = round(total, 2)
    res["unit"] = "s"
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
