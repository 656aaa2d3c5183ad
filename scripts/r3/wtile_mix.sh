#!/bin/bash
# Instruction mix of conv_wtile (stem 8-channel form vs conv2): SQ instruction counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
rm -rf gpurun_out/wmix
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_WAVES SQ_INSTS_SMEM \
  --kernel-trace --output-format csv -d gpurun_out/wmix -o pmc -- \
  python3 scripts/bench_conv_layers.py --batch 128 --reps 2 --only ${ONLY:-stem_s2d,conv2} > gpurun_out/wmix.log 2>&1
echo "pmc rc=$?"
python3 - "$(find gpurun_out/wmix -name "*counter_collection.csv" | head -1)" <<'PY'
import csv,sys
from collections import defaultdict
a=defaultdict(lambda: defaultdict(float)); n=defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    if 'wtile_kernel' in r['Kernel_Name']:
        k=r['Kernel_Name'][:45]; a[k][r['Counter_Name']]+=float(r['Counter_Value']); n[k].add(r['Dispatch_Id'])
for k,c in a.items():
    d=len(n[k]); print(k, d, {m:f"{v/d:.3e}" for m,v in c.items()})
PY
