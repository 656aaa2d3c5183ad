#!/bin/bash
# SQ counters of the fp8 and bf16 tile kernels on the 128^3 conv2 layer
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
rm -rf gpurun_out/f8pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_WAIT_INST_LDS \
  --kernel-trace --output-format csv -d gpurun_out/f8pmc -o pmc -- \
  python3 bench/f8_layers.py --batch 128 --reps 2 --layers ${L:-2} > gpurun_out/f8pmc.log 2>&1
echo "pmc rc=$?"
python3 - "$(find gpurun_out/f8pmc -name "*counter_collection.csv" | head -1)" <<'PY'
import csv,sys
from collections import defaultdict
a=defaultdict(lambda: defaultdict(float)); n=defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    if 'conv_tile_kernel' in r['Kernel_Name']:
        k=r['Kernel_Name'][:52]
        a[k][r['Counter_Name']]+=float(r['Counter_Value']); n[k].add(r['Dispatch_Id'])
for k,c in a.items():
    d=len(n[k]); print(k, d, {m:f"{v/d:.4e}" for m,v in sorted(c.items())})
PY
