#!/usr/bin/env python3
"""Tabulate the convergence-parity runs of bench/accuracy.py (native bf16 kernels vs the stock
PyTorch fp32 / bf16-autocast oracle, same init, same batches) from their JSON lines.

    python scripts/acc_summary.py gpurun_out > profiles/r6_convergence_parity.md
"""
import glob
import json
import os
import sys


def last_json(path):
    for line in reversed(open(path).read().splitlines()):
        if line.startswith("{"):
            try:
                return json.loads(line)
            except json.JSONDecodeError:
                return None
    return None


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    runs = {}
    for p in sorted(glob.glob(os.path.join(d, "acc_*_s*.log"))):
        r = last_json(p)
        if r is None:
            continue
        name = os.path.basename(p)[4:-4]                 # native_s0, torch32_s1, native_s3_repeat ...
        runs[name] = r
    impls = [("native", "native bf16 HIP kernels"), ("torch32", "stock PyTorch fp32"),
             ("torch16", "stock PyTorch bf16 autocast")]
    print("| seed | " + " | ".join(lbl for _, lbl in impls) + " |")
    print("|---|" + "---|" * len(impls))
    for s in range(4):
        cells = []
        for key, _ in impls:
            r = runs.get(f"{key}_s{s}")
            cells.append("-" if r is None else f"{r['value']:.4f}")
        print(f"| {s} | " + " | ".join(cells) + " |")
    print()
    for key, lbl in impls:
        vals = [runs[f"{key}_s{s}"]["value"] for s in range(4) if f"{key}_s{s}" in runs]
        if vals:
            print(f"* {lbl}: mean {sum(vals) / len(vals):.4f}, min {min(vals):.4f}, max {max(vals):.4f} "
                  f"over {len(vals)} seeds")
    print()
    print("Per-epoch held-out top-1:")
    print()
    for name, r in sorted(runs.items()):
        v = r.get("val_acc_per_epoch", [])
        sps = r.get("train_samples_per_s_per_epoch", [])
        extra = f", weights sha256 {r['weights_sha256']}" if "weights_sha256" in r else ""
        rate = f", {sum(sps) / len(sps):,.0f} samples/s" if sps else ""
        print(f"* `{name}`{extra}{rate}: " + " ".join(f"{x:.3f}" for x in v))
    a = runs.get("native_s3")
    for other, what in (("native_s3_repeat", "two processes, one box"), ("native_s3_box2", "another box")):
        b = runs.get(other)
        if a and b and "weights_sha256" in a:
            same = a["weights_sha256"] == b["weights_sha256"] and a["val_acc_per_epoch"] == b["val_acc_per_epoch"]
            print()
            print(f"Seed 3, {what}: weights {a['weights_sha256']} / {b['weights_sha256']} -- "
                  f"{'identical bits' if same else 'DIFFERENT'}.")


if __name__ == "__main__":
    main()
