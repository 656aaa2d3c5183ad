#!/bin/bash
# conv_tile schedule variants (FN_TILE_DBG 64: s_setprio 1 on the compute waves, 128: no per-fragment
# sched_barrier, 192: both) on conv2..conv4, fwd + dgrad
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for d in 0 64 128 192 0; do
  FN_TILE_DBG=$d timeout -k 10 120 python3 scripts/bench_conv_layers.py --batch 128 --reps 20 --only conv2,conv3,conv4 > gpurun_out/tsched_$d.log 2>&1 || { tail gpurun_out/tsched_$d.log; exit 1; }
  grep '^{' gpurun_out/tsched_$d.log | python3 -c "
import json,sys
for l in sys.stdin: r=json.loads(l); print('dbg $d', r['layer'], 'fwd', r['tile_fwd_us'], 'dgrad', r['tile_dgrad_us'])"
done
