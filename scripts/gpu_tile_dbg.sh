#!/bin/bash
# conv_tile experiment variants (FN_TILE_DBG, MT=8 plans only): 1 no B loads, 2 no A reads,
# 4 no halo DMA, 16 cycle stamps (barrier-A wait / job / tile end per workgroup, stderr)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in ${DBGS:-0 16 23}; do
  FN_TILE_DBG=$d timeout -k 10 120 python -u scripts/bench_conv_layers.py --batch 128 --reps 2 ${ONLY:+--only $ONLY} > gpurun_out/dbg_$d.log 2>&1 || exit $?
  echo "== dbg=$d"; grep -o '"layer": "[a-z0-9]*"\|"tile_fwd_us": [0-9.]*\|"tile_dgrad_us": [0-9.]*\|\[conv_tile stamps.*' gpurun_out/dbg_$d.log | head -60
done
exit 0
