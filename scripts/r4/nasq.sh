#!/bin/bash
# NAS workers per GPU vs HIP hardware queues per process (GPU_MAX_HW_QUEUES; the box default is 4)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "8 1" "8 2" "4 1" "8 4"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 300 python3 bench/search_throughput.py --candidates 32 --epochs 5 --dataset cifar \
    --graph on --workers-per-device $1 > gpurun_out/nasq_$1_$2.log 2>&1
  rc=$?; echo "workers $1 hwq $2 rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/nasq_$1_$2.log) $(grep -o '"trained": [0-9]*' gpurun_out/nasq_$1_$2.log)"
  [ $rc -eq 0 ] || exit $rc
done
