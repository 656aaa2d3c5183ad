#!/usr/bin/env python3
"""Per-kernel time summary of a rocprofv3 run_results.db (the SQLite output of ``rocprofv3
--kernel-trace`` without ``--output-format csv``): total ms, calls, mean us per kernel name.

    python scripts/rocpd_stats.py gpurun_out/prof/run_results.db [--top 20] [--md]
"""
import argparse
import sqlite3


def stats(path: str):
    con = sqlite3.connect(path)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    rows = con.execute(f"select {name}, count(*), sum(end - start) from kernels group by {name}").fetchall()
    return sorted(((n, c, t / 1e6) for n, c, t in rows), key=lambda r: -r[2])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=20)
    ap.add_argument("--md", action="store_true")
    a = ap.parse_args()
    rows = stats(a.db)
    tot = sum(r[2] for r in rows)
    print(f"total kernel ms {tot:.3f}")
    if a.md:
        print("| ms | % | calls | us/call | kernel |\n|---|---|---|---|---|")
    for n, c, t in rows[: a.top]:
        short = n if len(n) < 100 else n[:100]
        if a.md:
            print(f"| {t:.3f} | {100 * t / tot:.1f} | {c} | {1e3 * t / c:.1f} | `{short}` |")
        else:
            print(f"{t:9.3f} ms {100 * t / tot:5.1f}% {c:6d} {1e3 * t / c:9.1f} us  {short}")


if __name__ == "__main__":
    main()
