#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_small_kernels_gpu.py tests/test_dense_infer_gpu.py tests/test_determinism_gpu.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c3_tests.log 2>&1; rc=$?; tail -2 gpurun_out/c3_tests.log; grep -E "FAILED|ERROR" gpurun_out/c3_tests.log | head; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python scripts/diag_nas_step.py --list > gpurun_out/c3_nas.log 2>&1 || exit $?
tail -1 gpurun_out/c3_nas.log
bash scripts/gpu_tile_budget.sh
