#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_fp8_stem_gpu.py tests/test_kernels_gpu.py tests/test_conv_tile_gpu.py -k "fp8 or f8 or tile or stem" > gpurun_out/fp8q_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/fp8q_tests.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/fp8q_tests.log | head -20; exit $rc; }
PROF=1 ACC=0 bash scripts/r3/fp8.sh > /dev/null 2>&1; grep -v amdgpu gpurun_out/r3_fp8_1024.log
EP=16 bash scripts/r3/f8acc.sh
