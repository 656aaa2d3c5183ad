#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for f in 0 1; do
  FN_WTILE_FAKE=$f timeout -k 10 120 python3 scripts/bench_conv_layers.py --batch 128 --reps 5 --only conv2 > gpurun_out/wf.log 2>&1 || { tail gpurun_out/wf.log; exit 1; }
  grep '^{' gpurun_out/wf.log | python3 -c "
import json,sys
for l in sys.stdin: r=json.loads(l); print('fake $f', r['layer'], r['wtile_wgrad_us'])"
done
