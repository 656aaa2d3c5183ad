#!/bin/bash
# Training repeatability across processes: the same seed trained twice (bench/accuracy.py), the
# per-epoch losses printed side by side -- identical on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 200 python bench/accuracy.py --epochs 3 --train-per-class 400 --seed ${SEED:-3} > gpurun_out/rep_acc$r.log 2>&1 || exit $?
  grep -o '"loss_per_epoch": \[[^]]*\]' gpurun_out/rep_acc$r.log
done
