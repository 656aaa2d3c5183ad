"""Summarise a rocprofv3 kernel trace (``*_kernel_trace.csv``) into markdown.

Groups dispatches by (short kernel name, grid), reports per-step time, calls,
registers, scratch and LDS; usage:
``python scripts/prof_summary.py gpurun_out/prof/run_kernel_trace.csv --steps 7 > profiles/x.md``
(steps = timed + warmup steps the profiled bench ran, i.e. the number of
identical training steps in the trace).
"""
import argparse
import csv
import glob
import os
import re
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    n = name
    if n.startswith("_Z"):
        m = re.match(r"_Z\d+([A-Za-z_]\w*?)(I.*)?Ev", n)
        n = m.group(1) if m else n[:60]
    n = re.sub(r"\(.*$", "", n)
    n = n.replace("void ", "")
    if n.startswith("at::native::"):
        n = "torch:" + re.sub(r"<.*", "", n[len("at::native::"):])
    if n.startswith("Cijk_"):
        n = "hipblaslt:" + n.split("_MT")[1].split("_")[0] if "_MT" in n else "hipblaslt"
    return n[:80]


def rows_of(path: str):
    """Yield kernel-trace rows as CSV-style dicts from a ``*_kernel_trace.csv`` or a rocprofv3 ``.db``
    (the default output format; a directory is searched for either)."""
    if os.path.isdir(path):
        hits = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True) or \
            glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
        if not hits:
            raise SystemExit(f"no kernel trace under {path}")
        path = hits[0]
    if path.endswith(".db"):
        con = sqlite3.connect(path)
        q = ("select name, start, end, grid_x, workgroup_x, grid_y, grid_z, vgpr_count, accum_vgpr_count, "
             "scratch_size, lds_size from kernels")
        for n, st, en, gx, wx, gy, gz, v, a, sc, lds in con.execute(q):
            yield {"Kernel_Name": n, "Start_Timestamp": st, "End_Timestamp": en, "Grid_Size_X": gx,
                   "Workgroup_Size_X": wx, "Grid_Size_Y": gy, "Grid_Size_Z": gz, "VGPR_Count": v,
                   "Accum_VGPR_Count": a, "Scratch_Size": sc, "LDS_Block_Size": lds}
        return
    with open(path) as f:
        yield from csv.DictReader(f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    agg = defaultdict(lambda: {"ns": 0, "calls": 0, "vgpr": 0, "agpr": 0, "scratch": 0, "lds": 0})
    total = 0
    if True:
        for r in rows_of(a.trace):
            ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            grid = (int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
            k = (short(r["Kernel_Name"]), grid)
            e = agg[k]
            e["ns"] += ns
            e["calls"] += 1
            e["vgpr"], e["agpr"] = int(r["VGPR_Count"]), int(r["Accum_VGPR_Count"])
            e["scratch"], e["lds"] = int(r["Scratch_Size"]), int(r["LDS_Block_Size"])
            total += ns
    rows = sorted(agg.items(), key=lambda kv: -kv[1]["ns"])
    print(f"Total kernel time {total / 1e6:.2f} ms over {a.steps} steps = {total / 1e6 / a.steps:.3f} ms/step\n")
    print("| kernel | grid (WGs) | calls | ms/step | % | VGPR | AGPR | scratch | LDS |")
    print("|---|---|---|---|---|---|---|---|---|")
    for (name, grid), e in rows[:a.top]:
        print(f"| `{name}` | {grid[0]}x{grid[1]}x{grid[2]} | {e['calls']} | {e['ns'] / 1e6 / a.steps:.3f} | "
              f"{100 * e['ns'] / total:.1f} | {e['vgpr']} | {e['agpr']} | {e['scratch']} | {e['lds']} |")


if __name__ == "__main__":
    main()
