#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 bench/f8_layers.py --batch 128 > gpurun_out/f8q_0.log 2>&1 || { tail gpurun_out/f8q_0.log; exit 1; }
grep '^{' gpurun_out/f8q_0.log
FN_F8_DBG=16 timeout -k 10 200 python3 bench/f8_layers.py --batch 128 --no-bf16 --reps 2 > gpurun_out/f8q_16.log 2>&1 || { tail gpurun_out/f8q_16.log; exit 1; }
grep stamps gpurun_out/f8q_16.log | sort | uniq -c | sort -rn | head -4
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fp8" > gpurun_out/f8q_test.log 2>&1 || { tail -30 gpurun_out/f8q_test.log; exit 1; }
tail -1 gpurun_out/f8q_test.log
timeout -k 10 400 python3 bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 --steps 3 --warmup 1 > gpurun_out/f8q_1024.log 2>&1 || { tail gpurun_out/f8q_1024.log; exit 1; }
grep -v amdgpu.ids gpurun_out/f8q_1024.log | tail -4
