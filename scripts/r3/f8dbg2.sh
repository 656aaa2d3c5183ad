#!/bin/bash
# fp8 tile kernel: timing-only variants (3 = no weight loads + no halo reads, 7 = + no DMA) and cycle stamps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in 0 3 7 16; do
  FN_F8_DBG=$d timeout -k 10 200 python3 bench/f8_layers.py --batch 128 --no-bf16 --reps 3 > gpurun_out/f8d_$d.log 2>&1 || { tail gpurun_out/f8d_$d.log; exit 1; }
  grep '^{' gpurun_out/f8d_$d.log
done
grep stamps gpurun_out/f8d_16.log | sort | uniq -c | sort -rn | head -12
