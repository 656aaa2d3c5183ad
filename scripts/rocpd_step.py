#!/usr/bin/env python3
"""The last training step of a rocprofv3 kernel trace (SQLite ``*_results.db``) as a markdown
table in launch order: us, kernel, grid -- one step = the kernels from the last batch copy-in
(``copy2_kernel``) to the optimizer (``adam``) that follows it.

    python scripts/rocpd_step.py gpurun_out/f_prof/step_results.db [--marker copy2_kernel]
"""
import argparse
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="copy2_kernel")
    ap.add_argument("--end", default="adam")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = con.execute("select name, start, end, grid_x * grid_y * grid_z from kernels order by start").fetchall()
    first = max(i for i, r in enumerate(rows) if a.marker in r[0])
    last = max(i for i, r in enumerate(rows) if a.end in r[0])
    step = rows[first:last + 1] if last > first else rows[first:]
    tot = sum(e - s for _, s, e, _ in step) / 1e3
    span = (step[-1][2] - step[0][1]) / 1e3
    print("| us | kernel | grid |\n|---|---|---|")
    for n, s, e, g in step:
        short = re.sub(r"\(.*", "", n)[:90]
        print(f"| {(e - s) / 1e3:.1f} | `{short}` | {g} |")
    print(f"\nkernels {len(step)}; kernel total {tot:.1f} us; step span {span:.1f} us")


if __name__ == "__main__":
    main()
