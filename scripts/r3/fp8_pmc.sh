#!/bin/bash
# PMC counters of the fp8 128^3 inference forward (two passes, kernel-trace only)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA"
P2="FETCH_SIZE SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_INSTS_VALU"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1)); rm -rf gpurun_out/pmcf$i
  timeout -s KILL 200 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmcf$i -o pmc -- \
    python3 bench/infer_fp8.py --size 128 --batch 256 --chunk 256 --steps 1 --warmup 0 --only fp8 > gpurun_out/pmcf$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 scripts/pmc_summary.py gpurun_out/pmcf1/pmc_counter_collection.csv gpurun_out/pmcf2/pmc_counter_collection.csv --top 12 > gpurun_out/pmc_fp8.md
cat gpurun_out/pmc_fp8.md
