#!/bin/bash
# Whole GPU test suite (no -x: every failure is listed), the smoke test and the 1-GPU bench.
# Each step has its own time limit; an abort / crash / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n ${TAILN:-15} "gpurun_out/$name.log"
  return $rc
}
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
run pytest_gpu 1100 python -u -m pytest ${TESTS:-tests} -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
rc=$?; if fatal $rc; then exit $rc; fi
grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -40
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; if fatal $rc; then exit $rc; fi
run bench 300 python bench.py --steps 20 --warmup 5; rc=$?; if fatal $rc; then exit $rc; fi
exit 0
