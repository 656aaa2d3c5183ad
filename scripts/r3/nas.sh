#!/bin/bash
# NAS throughput at the census workload (32 candidates x 5 epochs, CIFAR-shaped), 1 and 4
# workers per GPU, plus a kernel census of a smaller run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python bench/search_throughput.py --candidates 32 --epochs 5 --dataset cifar --graph on > gpurun_out/nas_w1.log 2>&1 || { tail -20 gpurun_out/nas_w1.log; exit 1; }
grep '^{' gpurun_out/nas_w1.log
timeout -k 10 500 python bench/search_throughput.py --candidates 32 --epochs 5 --dataset cifar --graph on --workers-per-device 4 > gpurun_out/nas_w4.log 2>&1 || { tail -20 gpurun_out/nas_w4.log; exit 1; }
grep '^{' gpurun_out/nas_w4.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/nas_prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench/search_throughput.py" --candidates 8 --epochs 1 --dataset cifar --graph on > "$GRAFT_REPO_ROOT/gpurun_out/nas_prof.log" 2>&1 || exit 1
