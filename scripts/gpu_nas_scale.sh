#!/bin/bash
# NAS throughput vs run length: 4 and 8 workers per GPU over 32 and 128 CIFAR LeNet mutants x 5
# epochs (the timer includes spawning the workers: importing torch, HIP init, first kernels)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 32 128; do
  for w in 4 8; do
    timeout -k 10 400 python3 bench/search_throughput.py --candidates $n --epochs 5 --dataset cifar --graph on \
      --workers-per-device $w > gpurun_out/nasn_${n}_w$w.log 2>&1
    rc=$?; echo "candidates $n workers $w rc=$rc $(grep -o '"value": [0-9.]*\|"seconds": [0-9.]*' gpurun_out/nasn_${n}_w$w.log | tr '\n' ' ')"
    [ $rc -eq 0 ] || exit $rc
  done
done
