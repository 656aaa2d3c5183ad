#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
FN_CONV_TILE_NW=8 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv_tile_gpu.py > gpurun_out/t8_test.log 2>&1
rc=$?; tail -4 gpurun_out/t8_test.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/t8_test.log | head; exit $rc; }
for nw in 4 8; do
  FN_CONV_TILE_NW=$nw timeout -k 10 120 python3 scripts/bench_conv_layers.py --batch 128 --reps 5 --only stem_s2d,conv2,conv3,conv4 > gpurun_out/t8.log 2>&1 || { tail gpurun_out/t8.log; exit 1; }
  grep '^{' gpurun_out/t8.log | python3 -c "
import json,sys
for l in sys.stdin: r=json.loads(l); print('nw $nw', r['layer'], r.get('tile_fwd_us'), r.get('tile_dgrad_us'))"
done
