#!/bin/bash
# fp8 trained-model parity on the final fp8 path (two seeds)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for seed in ${SEEDS:-0 1}; do
  timeout -k 10 500 python3 bench/accuracy.py --epochs 16 --train-per-class 1000 --fp8 --seed $seed > gpurun_out/fpar_$seed.log 2>&1
  rc=$?; echo "seed $seed rc=$rc"; tail -3 gpurun_out/fpar_$seed.log | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
done
