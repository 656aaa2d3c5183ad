#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_determinism_gpu.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c4_tests.log 2>&1; rc=$?; tail -1 gpurun_out/c4_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/c4_tests.log | head; [ $rc -le 1 ] || exit $rc
FN_TILE_W8=1 timeout -k 10 300 python -u -m pytest tests/test_conv_tile_gpu.py tests/test_determinism_gpu.py tests/test_bnfuse_gpu.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c4_w8tests.log 2>&1; rc=$?; tail -1 gpurun_out/c4_w8tests.log; grep -E "^FAILED|^ERROR" gpurun_out/c4_w8tests.log | head; [ $rc -le 1 ] || exit $rc
for w in 0 1 0 1; do
  FN_TILE_W8=$w timeout -k 10 200 python -u scripts/bench_conv_layers.py --batch 128 --reps 5 --tile-only > gpurun_out/c4_layers_w$w.log 2>&1 || exit $?
  echo "w8=$w $(grep -o '"layer": "[a-z0-9_]*"\|"tile_[a-z_]*_us": [0-9.]*' gpurun_out/c4_layers_w$w.log | tr '\n' ' ')"
done
for w in 0 1 0 1; do
  FN_TILE_W8=$w timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/c4_bench_w$w.log 2>&1 || exit $?
  echo "bench w8=$w $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c4_bench_w$w.log)"
done
