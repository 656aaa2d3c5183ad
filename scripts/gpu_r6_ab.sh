#!/bin/bash
# Round 6: GPU tests of the kernels whose settled A/B switches were removed (dense, halo, fp8).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_small_kernels_gpu.py tests/test_fp8_stem_gpu.py \
  -q -m gpu --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -n 1 gpurun_out/ab_tests.log
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_bench.log 2>&1 || exit $?
tail -n 1 gpurun_out/ab_bench.log | cut -c1-140
