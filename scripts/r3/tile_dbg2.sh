#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for d in 0 32; do
  FN_TILE_DBG=$d timeout -k 10 120 python3 scripts/bench_conv_layers.py --batch 128 --reps 5 --only conv2,conv3 > gpurun_out/tdbg.log 2>&1 || { tail gpurun_out/tdbg.log; exit 1; }
  grep '^{' gpurun_out/tdbg.log | python3 -c "
import json,sys
for l in sys.stdin: r=json.loads(l); print('dbg $d', r['layer'], r['tile_fwd_us'], r['tile_dgrad_us'])"
done
