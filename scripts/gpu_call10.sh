#!/bin/bash
# FC1 kernels after the batched g / staging loads and the one-row-block forward rule: the FC
# micro-bench, the dense / conv GPU tests, then two training benches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python scripts/bench_fc_native.py --batch 128 --reps 50 > gpurun_out/c10_fc.log 2>&1 || exit $?
echo "fc $(tail -1 gpurun_out/c10_fc.log)"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_dense_infer_gpu.py -q -m gpu -k "dense or linear" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c10_tests.log 2>&1; rc=$?
tail -1 gpurun_out/c10_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/c10_tests.log | head
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/c10_bench$i.log 2>&1 || exit $?
  tail -1 gpurun_out/c10_bench$i.log | cut -c1-200
done
# robustness evaluation per candidate (CW + PGD + CLEVER with per-(sample, target) pools, 500 samples)
timeout -k 10 400 python bench/robustness.py > gpurun_out/c10_robust.log 2>&1 || exit $?
tail -3 gpurun_out/c10_robust.log | cut -c1-300
# NAS candidate step: launch list with the package frames behind each torch glue kernel
timeout -k 10 200 python scripts/diag_nas_step.py --list --stacks > gpurun_out/c10_nas_stacks.log 2>&1 || exit $?
tail -1 gpurun_out/c10_nas_stacks.log
