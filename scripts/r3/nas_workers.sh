#!/bin/bash
# NAS throughput at the census workload with 8 and 12 worker processes sharing one GPU
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in 8 12; do
  timeout -k 10 500 python bench/search_throughput.py --candidates 48 --epochs 5 --dataset cifar --graph on --workers-per-device $w > gpurun_out/nas_w$w.log 2>&1 || { tail -20 gpurun_out/nas_w$w.log; exit 1; }
  grep '^{' gpurun_out/nas_w$w.log
done
