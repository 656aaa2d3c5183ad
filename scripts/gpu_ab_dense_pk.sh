#!/bin/bash
# A/B of the K-permuted bf16-weight Dense forward (FN_DENSE_PK): its numerics tests, then the
# 128^3-inference FC1 micro-bench alternating, then the whole fp8 inference bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
FN_DENSE_PK=1 timeout -k 10 300 python -u -m pytest tests/test_dense_infer_gpu.py tests/test_kernels_gpu.py -k "dense or linear" \
  -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pk_tests.log 2>&1; rc=$?
tail -1 gpurun_out/pk_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/pk_tests.log | head
[ $rc -eq 0 ] || exit $rc
for p in 0 1 0 1; do
  FN_DENSE_PK=$p timeout -k 10 200 python scripts/bench_fc_infer.py > gpurun_out/pk_fc$p.log 2>&1 || exit $?
  echo "pk=$p $(tail -1 gpurun_out/pk_fc$p.log)"
done
for p in 0 1; do
  FN_DENSE_PK=$p timeout -k 10 300 python bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 > gpurun_out/pk_infer$p.log 2>&1 || exit $?
  echo "pk=$p $(grep -o '"value": [0-9.]*\|speedup[^,]*' gpurun_out/pk_infer$p.log | tr '\n' ' ')"
done
