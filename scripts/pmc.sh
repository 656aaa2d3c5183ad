#!/bin/bash
# PMC counters for the conv kernels (separate run: counters only with --kernel-trace/--stats).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
COUNTERS=${COUNTERS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"}
timeout -k 10 ${PTIME:-600} rocprofv3 --pmc $COUNTERS --kernel-trace --output-format csv -d gpurun_out/pmc -o pmc \
  -- python3 bench.py --steps 2 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/pmc_bench.log 2>&1
rc=$?
echo "pmc rc=$rc"; tail -2 gpurun_out/pmc_bench.log
ls gpurun_out/pmc
exit $rc
