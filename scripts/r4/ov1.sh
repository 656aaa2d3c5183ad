#!/bin/bash
# Round-4 (session 2) batch: weight gradients on a side stream (ops/overlap.py) -- tests,
# bench A/B (FN_WGRAD_STREAM=0/1, two runs each), kernel trace of the overlapped step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/ov_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ]; then tail -20 "gpurun_out/ov_$name.log"; exit $rc; fi
  return $rc
}
step tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_overlap_gpu.py
grep -E "passed|failed" gpurun_out/ov_tests.log | tail -2; grep -E "^FAILED|Error" gpurun_out/ov_tests.log | head -10
for i in 1 2; do
  for ws in 0 1; do
    FN_WGRAD_STREAM=$ws step bench_$ws 300 python3 bench.py --steps 30 --warmup 5
    echo "ws=$ws $(grep -o '"value": [0-9.]*' gpurun_out/ov_bench_$ws.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ov_bench_$ws.log)"
  done
done
rm -rf gpurun_out/prof_ov
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ov -o run -- \
  python3 bench.py --steps 5 --warmup 3
python3 scripts/step_breakdown.py gpurun_out/prof_ov/run_kernel_trace.csv --min-us 0 > gpurun_out/step_ov.md 2>&1 || true
tail -2 gpurun_out/step_ov.md
