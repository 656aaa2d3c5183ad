#!/bin/bash
# NAS throughput (32 CIFAR-shaped LeNet mutants x 5 epochs, hipGraph steps) at 1 / 4 / 8 workers
# per GPU, and the same at 4 workers with the CW + PGD robustness evaluation of every candidate.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in ${WORKERS:-1 4 8}; do
  timeout -k 10 300 python3 bench/search_throughput.py --candidates 32 --epochs 5 --dataset cifar --graph on \
    --workers-per-device $w > gpurun_out/nas_w$w.log 2>&1
  rc=$?; echo "workers $w rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/nas_w$w.log) $(grep -o '"trained": [0-9]*' gpurun_out/nas_w$w.log)"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python3 bench/search_throughput.py --candidates 32 --epochs 5 --dataset cifar --graph on \
  --workers-per-device 4 --attacks cw,pgd > gpurun_out/nas_w4_attacks.log 2>&1
rc=$?; echo "workers 4 + cw,pgd rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/nas_w4_attacks.log)"
exit $rc
