#!/usr/bin/env python3
"""Kernel sequence of ONE steady-state training step from a rocprofv3 kernel trace.

The step is the span between the last two ``adam_flat_kernel`` dispatches (the
optimizer ends every step); prints each kernel's duration and the step total.

    python scripts/step_breakdown.py gpurun_out/prof/run_kernel_trace.csv [--min-us 20]
"""
import argparse
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import short  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--min-us", type=float, default=20.0)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adam_flat" in r["Kernel_Name"]]
    if len(idx) < 2:
        raise SystemExit("need two optimizer steps in the trace")
    lo, hi = idx[-2], idx[-1]
    tot, small = 0.0, 0.0
    print("| us | kernel | grid |\n|---|---|---|")
    for r in rows[lo + 1:hi + 1]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        if d >= a.min_us:
            print(f"| {d:.1f} | `{short(r['Kernel_Name'])[:60]}` | {r.get('Grid_Size_X', r.get('Grid_Size', ''))} |")
        else:
            small += d
    span = (int(rows[hi]["End_Timestamp"]) - int(rows[lo]["End_Timestamp"])) / 1e3
    print(f"\nkernels < {a.min_us:g} us: {small:.1f} us; kernel total {tot:.1f} us; step span {span:.1f} us")


if __name__ == "__main__":
    main()
