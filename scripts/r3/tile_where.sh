#!/bin/bash
# Where the conv_tile k-loop time goes (timing-only DBG variants, wrong results), and the
# training step's PMC table (3 passes: issue/MFMA/LDS, HBM/instruction mix, L2 traffic).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in 0 1 2 4 3 7 32 16; do
  FN_TILE_DBG=$d timeout -k 10 120 python3 scripts/bench_conv_layers.py --batch 128 --reps 10 --only conv2 > gpurun_out/tdbg_$d.log 2>&1 || { tail gpurun_out/tdbg_$d.log; exit 1; }
  grep '^{' gpurun_out/tdbg_$d.log | python3 -c "
import json,sys
for l in sys.stdin: r=json.loads(l); print('dbg $d', r['layer'], 'fwd', r['tile_fwd_us'], 'dgrad', r['tile_dgrad_us'])"
  grep stamps gpurun_out/tdbg_$d.log | sort | uniq -c | head -4
done
bash scripts/gpu_pmc_bench.sh > gpurun_out/pmc_run.log 2>&1 || { tail -5 gpurun_out/pmc_run.log; exit 1; }
P3="TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
timeout -s KILL 150 rocprofv3 --pmc $P3 --kernel-trace --output-format csv -d gpurun_out/pmcb3 -o pmc -- \
    python3 bench.py --steps 2 --warmup 1 --graph off > gpurun_out/pmcb3.log 2>&1
echo "pmc pass 3 rc=$?"
