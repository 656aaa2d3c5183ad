#!/bin/bash
# Round-4 (session 2): dense dgrad / wgrad reuse of staged tiles, mask-epilogue trims -- tests,
# bench x2, kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/dn_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ]; then tail -20 "gpurun_out/dn_$name.log"; exit $rc; fi
  return $rc
}
step tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_bnfuse_gpu.py tests/test_small_kernels_gpu.py
grep -E "passed|failed" gpurun_out/dn_tests.log | tail -2; grep -E "^FAILED|Error" gpurun_out/dn_tests.log | head -10
[ -n "$(grep -E '^FAILED' gpurun_out/dn_tests.log)" ] && exit 1
for i in 1 2; do
  step bench 300 python3 bench.py --steps 30 --warmup 5
  echo "bench $(grep -o '"value": [0-9.]*' gpurun_out/dn_bench.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dn_bench.log)"
done
step dgstats 200 python3 scripts/r4/dgrad_stats_ab.py; grep layer gpurun_out/dn_dgstats.log
rm -rf gpurun_out/prof_dn
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dn -o run -- \
  python3 bench.py --steps 5 --warmup 3
python3 scripts/step_breakdown.py gpurun_out/prof_dn/run_kernel_trace.csv --min-us 0 > gpurun_out/step_dn.md 2>&1 || true
tail -2 gpurun_out/step_dn.md; grep -E "dense|conv_tile_kernel<8, 2, (2|4)" gpurun_out/step_dn.md
