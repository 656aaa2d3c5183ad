"""Aggregate a rocprofv3 --pmc counter CSV per (kernel, grid): derived utilisation ratios."""
import csv
import re
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402


def main(path):
    agg = defaultdict(lambda: defaultdict(float))
    with open(path) as f:
        for r in csv.DictReader(f):
            name = short(r.get("Kernel_Name", ""))
            grid = r.get("Grid_Size", r.get("Grid_Size_X", ""))
            key = (name, grid)
            agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
            agg[key]["_n"] += 1
    print("| kernel | grid | MFMA busy / busy | LDS active / busy | LDS bank-conflict / LDS active | wait LDS / wave cyc | wait any / wave cyc |")
    print("|---|---|---|---|---|---|---|")
    for (name, grid), c in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:20]:
        busy = c.get("SQ_BUSY_CYCLES", 0) or 1
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        lds = c.get("SQ_LDS_IDX_ACTIVE", 0) or 1
        print(f"| `{name}` | {grid} | {c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / busy:.3f} | "
              f"{c.get('SQ_LDS_IDX_ACTIVE', 0) / busy:.3f} | {c.get('SQ_LDS_BANK_CONFLICT', 0) / lds:.3f} | "
              f"{c.get('SQ_WAIT_INST_LDS', 0) / wc:.3f} | {c.get('SQ_WAIT_ANY', 0) / wc:.3f} |")


if __name__ == "__main__":
    main(sys.argv[1])
