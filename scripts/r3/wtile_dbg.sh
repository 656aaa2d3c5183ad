#!/bin/bash
# conv_wtile timing-only variants (FN_WTILE_DBG: 1 no next-x DMA, 4 no x halo DMA, 8 no dy DMA, 12 neither)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in 0 4 8 12; do
  echo "== dbg $d"
  FN_WTILE_DBG=$d timeout -k 10 120 python3 scripts/bench_conv_layers.py --batch 128 --reps 5 --only ${ONLY:-conv2,conv3,conv4} \
    > gpurun_out/wdbg_$d.log 2>&1 || { tail -5 gpurun_out/wdbg_$d.log; exit 1; }
  python3 -c "
import json,sys
for l in open('gpurun_out/wdbg_$d.log'):
    if l.startswith('{'):
        r=json.loads(l); print(r['layer'], {k:v for k,v in r.items() if k.endswith('_us')})
"
done
