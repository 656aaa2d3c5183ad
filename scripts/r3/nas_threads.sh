#!/bin/bash
# NAS throughput: trials as threads on their own HIP streams (one process) vs worker processes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in 4 8; do
  timeout -k 10 400 python bench/search_throughput.py --candidates 32 --epochs 5 --dataset cifar --graph on --mode threads --workers-per-device $w > gpurun_out/nas_thr$w.log 2>&1 || { tail -30 gpurun_out/nas_thr$w.log; exit 1; }
  grep '^{' gpurun_out/nas_thr$w.log | cut -c1-330
done
