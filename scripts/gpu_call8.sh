#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in 0 -1 0 -1; do
  FN_TILE_W8=$w timeout -k 10 200 python bench.py --model seg --steps 10 --warmup 3 > gpurun_out/c8_seg.log 2>&1 || exit $?
  echo "seg w8=[$w] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c8_seg.log)"
done
for w in 0 -1 0 -1; do
  FN_TILE_W8=$w timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/c8_cls.log 2>&1 || exit $?
  echo "cls w8=[$w] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c8_cls.log)"
done
timeout -k 10 300 python -u -m pytest tests/test_subpixel_gpu.py tests/test_determinism_gpu.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c8_tests.log 2>&1; rc=$?; tail -1 gpurun_out/c8_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/c8_tests.log | head; exit $rc
