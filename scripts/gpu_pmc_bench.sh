#!/bin/bash
# PMC counters of the training step (bench.py), one rocprofv3 run per counter pass
# (counters are collected with --kernel-trace only; every pass under its own KILL timeout).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA"
P2="FETCH_SIZE SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_INSTS_VALU"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  rm -rf gpurun_out/pmcb$i
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmcb$i -o pmc -- \
    python3 bench.py --steps 2 --warmup 1 --graph off ${BENCH_ARGS:-} > gpurun_out/pmcb$i.log 2>&1
  rc=$?
  echo "pmc pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 scripts/pmc_summary.py gpurun_out/pmcb1/pmc_counter_collection.csv gpurun_out/pmcb2/pmc_counter_collection.csv \
  --top 20 > gpurun_out/pmc_table.md
cat gpurun_out/pmc_table.md
