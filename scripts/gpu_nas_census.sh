#!/bin/bash
# Kernel census of NAS candidate training: rocprofv3 kernel trace + stats over 8 CIFAR LeNet
# mutants x 1 epoch (graph-replayed steps); summarise with scripts/rocpd_stats.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nas_census -o run -- \
  python3 bench/search_throughput.py --candidates 8 --epochs 1 --dataset cifar --graph on > gpurun_out/nas_census.log 2>&1 || exit $?
tail -2 gpurun_out/nas_census.log
