#!/bin/bash
# Round-4 (session 2): BN backward from the statistics identity (relu-mask dgrad epilogue,
# S = sum W . dW, no colstats pass) -- tests, bench A/B (FN_BN_IDENTITY=0/1), kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/id_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ]; then tail -20 "gpurun_out/id_$name.log"; exit $rc; fi
  return $rc
}
step tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_bnfuse_gpu.py tests/test_conv_tile_gpu.py tests/test_kernels_gpu.py tests/test_fp8_stem_gpu.py
grep -E "passed|failed" gpurun_out/id_tests.log | tail -2; grep -E "^FAILED|Error|rel err" gpurun_out/id_tests.log | head -10
[ -n "$(grep -E '^FAILED' gpurun_out/id_tests.log)" ] && exit 1
for i in 1 2; do
  for v in 0 1; do
    FN_BN_IDENTITY=$v step bench_$v 300 python3 bench.py --steps 30 --warmup 5
    echo "ident=$v $(grep -o '"value": [0-9.]*' gpurun_out/id_bench_$v.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/id_bench_$v.log) $(grep -o '"final_loss": [0-9.]*' gpurun_out/id_bench_$v.log)"
  done
done
rm -rf gpurun_out/prof_id
step dgstats 200 python3 scripts/r4/dgrad_stats_ab.py; grep layer gpurun_out/id_dgstats.log
FN_BN_IDENTITY=1 step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_id -o run -- \
  python3 bench.py --steps 5 --warmup 3
python3 scripts/step_breakdown.py gpurun_out/prof_id/run_kernel_trace.csv --min-us 0 > gpurun_out/step_id.md 2>&1 || true
tail -2 gpurun_out/step_id.md
FN_BN_IDENTITY=1 step seg 300 python3 bench.py --model seg --steps 10 --warmup 3
echo "seg $(grep -o '"value": [0-9.]*' gpurun_out/id_seg.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/id_seg.log)"
