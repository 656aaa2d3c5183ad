#!/bin/bash
# GPU check of the big-tile conv kernel: its tests, then per-layer timings vs conv_halo.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 300 python -u -m pytest tests/test_conv_tile_gpu.py -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/tile_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 15 gpurun_out/tile_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_conv_layers.py --batch 128 --reps 10 > gpurun_out/tile_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; cat gpurun_out/tile_bench.log | cut -c1-600
exit $rc
