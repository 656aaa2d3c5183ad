#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for pf in 4 20; do for d in 0 12; do
  echo "== pf $pf dbg $d"
  FN_WTILE_PF=$pf FN_WTILE_DBG=$d timeout -k 10 120 python3 scripts/bench_conv_layers.py --batch 128 --reps 5 --only conv2 \
    > gpurun_out/wpf.log 2>&1 || { tail -5 gpurun_out/wpf.log; exit 1; }
  grep '^{' gpurun_out/wpf.log | python3 -c "
import json,sys
for l in sys.stdin: r=json.loads(l); print(r['layer'], r['wtile_wgrad_us'])"
done; done
