#!/bin/bash
# GPU-box check: kernel numerics tests, smoke, native bench, torch baseline bench.
# Every GPU step runs under its own timeout; a crash / timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-10}
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 12 "gpurun_out/$name.log"
  return $rc
}
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  run pytest_gpu 900 python -u -m pytest ${TESTS:-tests} -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider; rc=$?
  if fatal $rc; then exit $rc; fi
fi
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; if fatal $rc; then exit $rc; fi
run bench_native 600 python bench.py --steps "$STEPS" --warmup 3; rc=$?; if fatal $rc; then exit $rc; fi
if [ "${SKIP_TORCH:-0}" != "1" ]; then
  run bench_torch 600 python bench.py --impl torch --steps "$STEPS" --warmup 3; rc=$?; if fatal $rc; then exit $rc; fi
fi
exit 0
