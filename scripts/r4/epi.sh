#!/bin/bash
# Round-4 (session 2): packed-pair conv_tile epilogue -- conv / BN tests, stem timing stamps,
# bench x2, kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/epi_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ]; then tail -20 "gpurun_out/epi_$name.log"; exit $rc; fi
  return $rc
}
step tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_tile_gpu.py tests/test_bnfuse_gpu.py tests/test_fp8_stem_gpu.py tests/test_kernels_gpu.py
grep -E "passed|failed" gpurun_out/epi_tests.log | tail -2; grep -E "^FAILED|Error" gpurun_out/epi_tests.log | head -10
[ -n "$(grep -E '^FAILED' gpurun_out/epi_tests.log)" ] && exit 1
for d in 0 16; do
  FN_TILE_DBG=$d step stem_$d 120 python3 scripts/bench_conv_layers.py --batch 128 --reps 10 --only stem_s2d,conv2
  echo "dbg=$d"; grep -o '"layer": "[a-z0-9_]*"\|"tile_fwd_us": [0-9.]*\|"tile_dgrad_us": [0-9.]*' gpurun_out/epi_stem_$d.log | paste - - - ; grep -h "wave0" gpurun_out/epi_stem_$d.log | head -2
done
for i in 1 2; do
  step bench 300 python3 bench.py --steps 30 --warmup 5
  echo "bench $(grep -o '"value": [0-9.]*' gpurun_out/epi_bench.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/epi_bench.log)"
done
step dgstats 200 python3 scripts/r4/dgrad_stats_ab.py; cat gpurun_out/epi_dgstats.log | grep layer
rm -rf gpurun_out/prof_epi
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_epi -o run -- \
  python3 bench.py --steps 5 --warmup 3
python3 scripts/step_breakdown.py gpurun_out/prof_epi/run_kernel_trace.csv --min-us 0 > gpurun_out/step_epi.md 2>&1 || true
tail -2 gpurun_out/step_epi.md
