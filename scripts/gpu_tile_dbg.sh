#!/bin/bash
# conv_tile experiment variants on conv2 forward/dgrad (timing only)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in 0 1 2 4 3 7; do
  FN_TILE_DBG=$d timeout -k 10 120 python -u scripts/bench_conv_layers.py --batch 128 --reps 10 --only conv2 > gpurun_out/dbg_$d.log 2>&1 || exit $?
  echo "dbg=$d $(grep -o '"tile_fwd_us": [0-9.]*' gpurun_out/dbg_$d.log) $(grep -o '"tile_dgrad_us": [0-9.]*' gpurun_out/dbg_$d.log)"
done
exit 0
