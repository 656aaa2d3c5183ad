#!/bin/bash
# Robustness as a GPU path: 500-sample CW + PGD + CLEVER for a CIFAR LeNet-5 candidate (seconds
# per metric), the launch census of that evaluation (no weight-gradient entry points), and NAS
# candidates/hour with robustness included.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 bench/robustness.py --set-size 500 --clever 500 --metrics clever,pgd,cw \
  > gpurun_out/robust_500.log 2>&1 || { tail gpurun_out/robust_500.log; exit 1; }
grep '^{' gpurun_out/robust_500.log
timeout -k 10 300 python3 bench/robustness.py --set-size 100 --clever 20 --metrics clever,pgd,cw --census \
  > gpurun_out/robust_census.log 2>&1 || { tail gpurun_out/robust_census.log; exit 1; }
grep '^{' gpurun_out/robust_census.log
for w in 1 4; do
  timeout -k 10 600 python3 bench/search_throughput.py --candidates 16 --epochs 3 --dataset cifar --graph on \
    --workers-per-device $w --attacks cw,pgd --robustness-set 500 > gpurun_out/nas_attacks_w$w.log 2>&1 || { tail gpurun_out/nas_attacks_w$w.log; exit 1; }
  grep '^{' gpurun_out/nas_attacks_w$w.log
done
