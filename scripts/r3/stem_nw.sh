#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for nw in 4 8 4 8; do
  FN_CONV_TILE_NW=$nw timeout -k 10 120 python3 scripts/bench_conv_layers.py --batch 128 --reps 20 --only stem_s2d > gpurun_out/stem_nw$nw.log 2>&1 || { tail gpurun_out/stem_nw$nw.log; exit 1; }
  grep '^{' gpurun_out/stem_nw$nw.log | python3 -c "
import json,sys
for l in sys.stdin: r=json.loads(l); print('nw $nw', r['layer'], 'fwd', r['tile_fwd_us'], 'dgrad', r.get('tile_dgrad_us'), r['tile_fwd_plan'][:80])"
done
