#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
# training repeatability across processes: the same seed twice
for r in 1 2; do
  timeout -k 10 200 python bench/accuracy.py --epochs 3 --train-per-class 400 --seed 3 > gpurun_out/c5_acc$r.log 2>&1 || exit $?
  grep -o '"loss_per_epoch": \[[^]]*\]' gpurun_out/c5_acc$r.log
done
bash scripts/gpu_nas.sh
