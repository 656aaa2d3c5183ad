#!/bin/bash
# Round-4 (session 2): memory-bound BN / pool passes (pool moments with all window loads in
# flight, 32-bit index math, resident-sized colstats grids) -- tests, bench x2, kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/mb_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ]; then tail -20 "gpurun_out/mb_$name.log"; exit $rc; fi
  return $rc
}
step tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_bnfuse_gpu.py tests/test_kernels_gpu.py -k "bn or pool or batchnorm or featurenet"
grep -E "passed|failed" gpurun_out/mb_tests.log | tail -2; grep -E "^FAILED|Error" gpurun_out/mb_tests.log | head -10
for i in 1 2; do
  step bench 300 python3 bench.py --steps 30 --warmup 5
  echo "bench $(grep -o '"value": [0-9.]*' gpurun_out/mb_bench.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/mb_bench.log)"
done
rm -rf gpurun_out/prof_mb
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mb -o run -- \
  python3 bench.py --steps 5 --warmup 3
python3 scripts/step_breakdown.py gpurun_out/prof_mb/run_kernel_trace.csv --min-us 0 > gpurun_out/step_mb.md 2>&1 || true
tail -2 gpurun_out/step_mb.md
