#!/bin/bash
# conv_tile per-phase budget: builds the experiment instances ON THE BOX (the in-tree library stays
# the production build), then times conv2-4 fwd / dgrad / masked dgrad per FN_TILE_DBG variant
# (0 production, 16 cycle stamps, 1 no weight loads, 2 no halo reads, 4 no halo DMA, 8 no output
# stores, 32 constant tap offsets, 64 compute-wave priority, 128 free k-step scheduling) and runs
# two rocprofv3 PMC passes over the production kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
FN_BUILD_EXPERIMENTS=1 timeout -k 10 600 python -m featurenet_amd._build > gpurun_out/build_exp.log 2>&1 || { tail gpurun_out/build_exp.log; exit 1; }
for d in ${DBGS:-0 1 2 3 4 8 32 64 128}; do
  FN_TILE_DBG=$d timeout -k 10 180 python -u scripts/bench_conv_layers.py --batch 128 --reps 3 --tile-only \
    > gpurun_out/budget_$d.log 2>&1 || { echo "dbg $d failed"; tail -5 gpurun_out/budget_$d.log; exit 1; }
  [ "$d" = 0 ] && cp gpurun_out/budget_0.log gpurun_out/budget_base.log
  echo "== dbg=$d"
  grep -o '"layer": "[a-z0-9_]*"\|"tile_[a-z_]*_us": [0-9.]*\|\[conv_tile stamps.*' gpurun_out/budget_$d.log | tr '\n' ' '
  echo
done
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/budget_pmc$i -o pmc -- \
    python3 scripts/bench_conv_layers.py --batch 128 --reps 2 --tile-only > gpurun_out/budget_pmc$i.log 2>&1
  echo "pmc pass $i rc=$?"
done
exit 0
