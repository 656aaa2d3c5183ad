#!/bin/bash
# PMC A/B of the conv k-loops: conv_tile (16x16x32) vs conv_tile32 (32x32x16) in the training
# step (bench.py --graph off): MFMA / LDS utilisation, bank conflicts, waits, and the effective
# clock (GRBM_GUI_ACTIVE / 8 / wall).  One rocprofv3 pass per counter set, each under its own
# KILL timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA"
P2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
for m in 0 1; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    rm -rf gpurun_out/m32pmc_${m}_$i
    FN_TILE_M32=$m timeout -s KILL 150 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/m32pmc_${m}_$i -o pmc -- \
      python3 bench.py --steps 2 --warmup 1 --graph off > gpurun_out/m32pmc_${m}_$i.log 2>&1
    rc=$?
    echo "m32=$m pmc pass $i rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
  python3 scripts/pmc_summary.py gpurun_out/m32pmc_${m}_1/pmc_counter_collection.csv gpurun_out/m32pmc_${m}_2/pmc_counter_collection.csv \
    --top 8 > gpurun_out/m32pmc_$m.md
  cat gpurun_out/m32pmc_$m.md
done
