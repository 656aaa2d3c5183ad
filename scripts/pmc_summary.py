"""Aggregate a rocprofv3 --pmc counter CSV per (kernel, grid) into utilisation ratios.

Ratios are normalised by the kernel's own duration (End-Start of each dispatch)
at an assumed shader clock (``--ghz``, profiled runs hold ~2.0-2.1 GHz) over
all 256 CUs / 1024 SIMDs of an MI355X:

* MFMA util   = SQ_VALU_MFMA_BUSY_CYCLES / (cycles x 1024 SIMDs)
* LDS util    = SQ_LDS_IDX_ACTIVE / (cycles x 256 CUs)
* bank confl. = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
* wait / wave = SQ_WAIT_ANY / SQ_WAVE_CYCLES  (waves parked on s_waitcnt / barrier)
* stall/wave  = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (issue stalls)
* HBM GB/s    = FETCH_SIZE (KB read from HBM via the TCC/EA) / kernel time, when collected
* with a second pass holding them: effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel time,
  LDS and VALU instructions per MFMA, LDS-issue stall share (SQ_WAIT_INST_LDS / wave cycles)

Several CSVs (one per counter pass of the same program) are merged per (kernel, grid);
times come from the first pass.

usage: python scripts/pmc_summary.py pass1/pmc_counter_collection.csv [pass2/...csv] [--ghz 2.1]
"""
import argparse
import csv
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--ghz", type=float, default=2.1)
    ap.add_argument("--top", type=int, default=16)
    a = ap.parse_args()
    agg = defaultdict(lambda: defaultdict(float))
    durs = defaultdict(dict)
    for i, path in enumerate(a.csv):
        with open(path) as f:
            for r in csv.DictReader(f):
                key = (short(r.get("Kernel_Name", "")), r.get("Grid_Size", ""))
                agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
                if i == 0:
                    durs[key][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    print(f"Counters normalised at {a.ghz} GHz over 1024 SIMDs / 256 CUs.\n")
    extra = any("GRBM_GUI_ACTIVE" in c for c in agg.values())
    print("| kernel | grid (threads) | time ms | MFMA util | LDS util | bank conflict / LDS cyc | wait / wave cyc | "
          "issue stall / wave cyc | HBM read GB/s |" + (" clock GHz | LDS inst / MFMA | VALU inst / MFMA | "
                                                         "LDS stall / wave cyc |" if extra else ""))
    print("|---|---|---|---|---|---|---|---|---|" + ("---|---|---|---|" if extra else ""))
    rows = sorted((kv for kv in agg.items() if kv[0] in durs), key=lambda kv: -sum(durs[kv[0]].values()))[: a.top]
    for (name, grid), c in rows:
        ns = sum(durs[(name, grid)].values())
        cyc = max(ns * a.ghz, 1.0)
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        lds = c.get("SQ_LDS_IDX_ACTIVE", 0)
        print(f"| `{name}` | {grid} | {ns / 1e6:.3f} | {c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (cyc * 1024):.3f} | "
              f"{lds / (cyc * 256):.3f} | {c.get('SQ_LDS_BANK_CONFLICT', 0) / max(lds, 1):.3f} | "
              f"{c.get('SQ_WAIT_ANY', 0) / wc:.3f} | {c.get('SQ_WAIT_INST_ANY', 0) / wc:.3f} | "
              f"{(c['FETCH_SIZE'] * 1024 / ns if 'FETCH_SIZE' in c else float('nan')):.0f} |" +
              (f" {c.get('GRBM_GUI_ACTIVE', 0) / 8 / ns:.2f} | "
               f"{c.get('SQ_INSTS_LDS', 0) / max(c.get('SQ_INSTS_MFMA', 0), 1):.2f} | "
               f"{c.get('SQ_INSTS_VALU', 0) / max(c.get('SQ_INSTS_MFMA', 0), 1):.2f} | "
               f"{c.get('SQ_WAIT_INST_LDS', 0) / wc:.3f} |" if extra else ""))


if __name__ == "__main__":
    main()
