#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
FN_WTILE_NW=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_wtile_gpu.py -p no:cacheprovider > gpurun_out/wt8_test.log 2>&1
rc=$?; tail -5 gpurun_out/wt8_test.log; [ $rc -eq 0 ] || exit $rc
for nw in 4 8; do
  FN_WTILE_NW=$nw timeout -k 10 120 python3 scripts/bench_conv_layers.py --batch 128 --reps 5 --only conv2,conv3,conv4 > gpurun_out/wt8.log 2>&1 || { tail gpurun_out/wt8.log; exit 1; }
  grep '^{' gpurun_out/wt8.log | python3 -c "
import json,sys
for l in sys.stdin: r=json.loads(l); print('nw $nw', r['layer'], r['wtile_wgrad_us'], r['halo_wgrad_us'])"
done
