#!/bin/bash
# one-launch batch copy-in: tests, bench x2, step trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_copy_in_gpu.py tests/test_bench_contract.py -x -q -m gpu --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/ci_test.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/ci_test.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 > gpurun_out/ci_bench.log 2>&1 || exit 1
  echo "bench $(grep -o '"value": [0-9.]*' gpurun_out/ci_bench.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ci_bench.log)"
done
rm -rf gpurun_out/prof_ci
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_ci -o run -- \
  python3 bench.py --steps 5 --warmup 3 > gpurun_out/ci_prof.log 2>&1 || exit 1
python3 scripts/step_breakdown.py gpurun_out/prof_ci/run_kernel_trace.csv --min-us 0 > gpurun_out/step_ci.md 2>&1
tail -1 gpurun_out/step_ci.md; head -8 gpurun_out/step_ci.md
