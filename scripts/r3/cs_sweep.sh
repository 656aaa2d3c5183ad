#!/bin/bash
# conv_tile plan sweep: forced channel-slice width per layer (FN_TILE_CS) vs the planner's choice
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for rk in 0 1 2 3 0; do
  FN_TILE_PLAN_RANK=$rk timeout -k 10 150 python3 scripts/bench_conv_layers.py --batch 128 --reps 20 --only conv2,conv3,conv4 > gpurun_out/rk_$rk.log 2>&1 || { tail -5 gpurun_out/rk_$rk.log; continue; }
  grep '^{' gpurun_out/rk_$rk.log | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print('rk $rk', r['layer'], 'fwd', r.get('tile_fwd_us'), 'dgrad', r.get('tile_dgrad_us'), '|', r['tile_fwd_plan'][9:60], '|', r['tile_dgrad_plan'][9:60])"
done
