#!/bin/bash
# Round 6: the stock PyTorch oracle of the convergence-parity table (bench/accuracy.py --impl torch,
# MIOpen find mode, channels-last; same init and batch order as the native runs).
#   bash scripts/gpu_r6_acc3.sh fp32 0 1      # dtype, seeds
# (MIOpen's find database persists across the processes of one box: the first seed pays the search)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
dt=$1; shift
tag=$([ "$dt" = fp32 ] && echo torch32 || echo torch16)
for s in "$@"; do
  timeout -k 10 560 python -u bench/accuracy.py --impl torch --torch-dtype $dt --epochs 16 --train-per-class 1000 \
    --seed $s > gpurun_out/acc_${tag}_s$s.log 2>&1 || exit $?
  tail -n 1 gpurun_out/acc_${tag}_s$s.log | cut -c1-220
done
