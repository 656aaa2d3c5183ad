"""Kernel census of a NAS candidate run (rocprofv3 --kernel-trace --stats directory): time by
origin (gather kernels, torch glue, D2D copies, other native) and the top kernels.

    python scripts/r4/nas_census.py gpurun_out/sprof_b7
"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from prof_summary import short  # noqa: E402


def origin(name: str, raw: str) -> str:
    if "copyBuffer" in raw or "fillBuffer" in raw:
        return "copy / fill (rocclr)"
    if name.startswith("torch") or "at::" in raw:
        return "torch glue"
    if "igemm" in raw:
        return "igemm gather kernels"
    return "other native"


def main():
    d = sys.argv[1]
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    cat = collections.defaultdict(float)
    calls = collections.Counter()
    out = []
    for r in rows:
        n = short(r["Name"])
        t = float(r["TotalDurationNs"]) / 1e6
        k = origin(n, r["Name"])
        cat[k] += t
        calls[k] += int(r["Calls"])
        out.append((t, int(r["Calls"]), n))
    tot = sum(cat.values())
    print(f"total kernel time {tot:.1f} ms, {sum(calls.values())} launches\n")
    print("| origin | ms | % | calls |\n|---|---|---|---|")
    for k, v in sorted(cat.items(), key=lambda kv: -kv[1]):
        print(f"| {k} | {v:.1f} | {100 * v / tot:.1f} | {calls[k]} |")
    print("\n| ms | calls | kernel |\n|---|---|---|")
    for t, c, n in sorted(out, reverse=True)[:30]:
        print(f"| {t:.1f} | {c} | `{n[:90]}` |")


if __name__ == "__main__":
    main()
