#!/bin/bash
# fp8 vs bf16 per-layer times at 128^3 and the fp8 kernel's timing-only variants
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
B=${B:-128}
timeout -k 10 200 python3 bench/f8_layers.py --batch $B > gpurun_out/f8l_0.log 2>&1 || { tail gpurun_out/f8l_0.log; exit 1; }
grep '^{' gpurun_out/f8l_0.log
for d in ${DBGS:-1 2 4}; do
  FN_F8_DBG=$d timeout -k 10 200 python3 bench/f8_layers.py --batch $B --no-bf16 > gpurun_out/f8l_$d.log 2>&1 || { tail gpurun_out/f8l_$d.log; exit 1; }
  grep '^{' gpurun_out/f8l_$d.log
done
