#!/bin/bash
# Focused GPU-box check: selected GPU tests (TESTS), the 1-GPU bench and a rocprofv3 kernel
# trace of it (step breakdown).  Every GPU step has its own time limit; a crash, abort or
# timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 8 "gpurun_out/$name.log"
  return $rc
}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
if [ -n "${TESTS:-}" ]; then
  step pytest_sel 600 python -u -m pytest $TESTS -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
  rc=$?; ok $rc || exit $rc
fi
step bench 300 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-}; rc=$?; ok $rc || exit $rc
if [ "${SKIP_PROF:-0}" != "1" ]; then
  step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 5 --warmup 2 ${BENCH_ARGS:-}
  rc=$?; ok $rc || exit $rc
  python3 scripts/step_breakdown.py gpurun_out/prof/run_kernel_trace.csv --min-us 0 > gpurun_out/step.md 2>&1
  tail -n 3 gpurun_out/step.md
fi
exit 0
