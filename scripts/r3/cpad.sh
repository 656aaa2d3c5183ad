#!/bin/bash
# channel-padded NAS conv path: GPU numerics, search-space shapes, NAS throughput
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "channel_padded or search_space or conv_fwd_bwd" > gpurun_out/cpad_test.log 2>&1 || { tail -30 gpurun_out/cpad_test.log; exit 1; }
tail -2 gpurun_out/cpad_test.log
timeout -k 10 400 python3 bench/search_throughput.py --candidates 16 --epochs 2 --dataset cifar --graph on > gpurun_out/nas_cp.log 2>&1 || { tail -20 gpurun_out/nas_cp.log; exit 1; }
grep '^{' gpurun_out/nas_cp.log
