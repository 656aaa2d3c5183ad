#!/bin/bash
# Round 6: the trained-model fp8 agreement test (and the rest of the block-scaled fp8 tests).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fp8_block_gpu.py -v -s -m gpu --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/z_tests.log 2>&1 || { tail -30 gpurun_out/z_tests.log; exit 1; }
grep -E "PASS|FAIL|bf16 top-1" gpurun_out/z_tests.log | tail -12
