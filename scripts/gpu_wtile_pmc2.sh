#!/bin/bash
# conv_wtile vs conv_halo wgrad: SQ counters (MFMA busy, LDS active / bank conflicts, waits) on the layer bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/wpmc2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS \
  --kernel-trace --output-format csv -d gpurun_out/wpmc2 -o pmc -- \
  python3 scripts/bench_conv_layers.py --batch 128 --reps 2 --only conv2,conv3,conv4 > gpurun_out/wpmc2.log 2>&1
echo "pmc rc=$?"
python3 scripts/pmc_summary.py $(find gpurun_out/wpmc2 -name "*counter_collection.csv" | head -1) --top 12
