#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 0 1 0 1; do
  FN_DENSE_NCW=$n timeout -k 10 120 python scripts/bench_fc_native.py --batch 128 --reps 50 > gpurun_out/c9_fc$n.log 2>&1 || exit $?
  echo "ncw=$n $(tail -1 gpurun_out/c9_fc$n.log)"
done
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -k "conv_fwd_bwd or dense" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c9_tests.log 2>&1; rc=$?; tail -1 gpurun_out/c9_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/c9_tests.log | head; exit $rc
