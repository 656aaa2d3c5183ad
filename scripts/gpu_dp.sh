#!/bin/bash
# GPU-box check of the data-parallel path on one MI355X:
#   1. the GPU test suite (incl. the 2-rank DP gradient test),
#   2. bench.py (1 GPU) and bench.py --force-allreduce (single-rank RCCL communicator:
#      the bucketed all-reduces are issued from the gradient hooks through RCCL),
#   3. a rocprofv3 kernel trace of the forced-all-reduce run (RCCL kernels vs conv kernels).
# Every GPU step has its own time limit; a crash, abort or timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-20}
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 6 "gpurun_out/$name.log"
  return $rc
}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = test failures: keep going; anything else stops
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  step pytest_gpu 900 python -u -m pytest ${TESTS:-tests} -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
  rc=$?; ok $rc || exit $rc
fi
step bench_native 300 python bench.py --steps "$STEPS" --warmup 5; rc=$?; ok $rc || exit $rc
step bench_forced_rccl 300 python bench.py --steps "$STEPS" --warmup 5 --force-allreduce; rc=$?; ok $rc || exit $rc
if [ "${SKIP_PROF:-0}" != "1" ]; then
  step prof_rccl 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rccl -o run -- \
    python3 bench.py --steps 5 --warmup 2 --force-allreduce --bucket-mb 4
  rc=$?; ok $rc || exit $rc
fi
exit 0
