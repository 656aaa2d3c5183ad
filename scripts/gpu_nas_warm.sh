#!/bin/bash
# NAS throughput with a persistent worker pool: 32 CIFAR LeNet mutants x 5 epochs at 4 and 8
# workers per GPU, cold (the clock includes starting the workers) and warm (--warm: the pool
# started before the clock, the steady state of a multi-generation search)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in 4 8; do
  for warm in "" "--warm"; do
    timeout -k 10 400 python3 bench/search_throughput.py --candidates 32 --epochs 5 --dataset cifar --graph on \
      --workers-per-device $w $warm > gpurun_out/nasw_${w}${warm}.log 2>&1
    rc=$?; echo "workers $w ${warm:-cold} rc=$rc $(grep -o '"value": [0-9.]*\|"seconds": [0-9.]*\|"trained": [0-9]*' gpurun_out/nasw_${w}${warm}.log | tr '\n' ' ')"
    [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 400 python3 bench/search_throughput.py --candidates 32 --epochs 5 --dataset cifar --graph on \
  --workers-per-device 4 --warm --attacks cw,pgd > gpurun_out/nasw_4_attacks.log 2>&1
rc=$?; echo "workers 4 warm + cw,pgd rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/nasw_4_attacks.log)"
exit $rc
