#!/bin/bash
# conv_tile: tests, layer bench, then one PMC pass over the layer bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_tile.sh || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d gpurun_out/pmc_tile -o pmc -- python3 scripts/bench_conv_layers.py --batch 128 --reps 2 > gpurun_out/pmc_tile.log 2>&1
echo "pmc rc=$?"
exit 0
