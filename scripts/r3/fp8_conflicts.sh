#!/bin/bash
# Where the fp8 conv_tile LDS bank conflicts come from: one counter pass per timing-only
# variant (FN_F8_DBG: 0 production, 2 no halo fragment reads, 4 no halo DMA, 1 no weight loads)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA"
for D in 0 2 4 1; do
  rm -rf gpurun_out/f8c$D
  export FN_F8_DBG=$D
  timeout -s KILL 200 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d gpurun_out/f8c$D -o pmc -- \
    python3 bench/infer_fp8.py --size 128 --batch 256 --chunk 256 --steps 1 --warmup 0 --only fp8 > gpurun_out/f8c$D.log 2>&1
  rc=$?; echo "dbg $D rc=$rc"; [ $rc -eq 0 ] || exit $rc
  echo "== FN_F8_DBG=$D" >> gpurun_out/f8c.md
  python3 scripts/pmc_summary.py gpurun_out/f8c$D/pmc_counter_collection.csv --top 2 >> gpurun_out/f8c.md
done
unset FN_F8_DBG
cat gpurun_out/f8c.md
