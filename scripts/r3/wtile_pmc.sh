#!/bin/bash
# SQ counters of conv_wtile on conv2 (full run and DMA-free timing variant)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for d in 0 12; do
rm -rf gpurun_out/wpmc_$d
FN_WTILE_DBG=$d timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS \
  --kernel-trace --output-format csv -d gpurun_out/wpmc_$d -o pmc -- \
  python3 scripts/bench_conv_layers.py --batch 128 --reps 2 --only ${ONLY:-conv2} > gpurun_out/wpmc_$d.log 2>&1
echo "pmc rc=$?"
python3 scripts/pmc_summary.py $(find gpurun_out/wpmc_$d -name "*counter_collection.csv" | head -1) --top 8
python3 - "$(find gpurun_out/wpmc_$d -name "*counter_collection.csv" | head -1)" <<'PY'
import csv,sys
from collections import defaultdict
a=defaultdict(lambda: defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    if 'wtile_kernel' in r['Kernel_Name']:
        a[r['Kernel_Name'][:40]][r['Counter_Name']]+=float(r['Counter_Value'])
for k,c in a.items(): print(k, {n:f"{v:.3e}" for n,v in c.items()})
PY
done
