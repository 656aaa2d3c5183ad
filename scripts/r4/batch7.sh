#!/bin/bash
# Round-4 batch 7: int8 diagnostics, GPU tests of the changed kernels (conv tile epilogue
# statistics in registers, BWS-16 removal, NAS gather wgrad fusions, dense fusions), stem layer
# times, training bench, step trace, NAS throughput + kernel census.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/b7_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ]; then tail -20 "gpurun_out/b7_$name.log"; exit $rc; fi
  return $rc
}
step i8dbg 120 python3 scripts/r4/i8_debug.py; grep -v amdgpu.ids gpurun_out/b7_i8dbg.log | tail -20
step tests 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_tile_gpu.py tests/test_bnfuse_gpu.py tests/test_kernels_gpu.py tests/test_subpixel_gpu.py
grep -E "passed|failed" gpurun_out/b7_tests.log | tail -2; grep -E "^FAILED|Error:" gpurun_out/b7_tests.log | head -10
step layers 200 python -u scripts/bench_conv_layers.py --batch 128 --reps 10
grep -o '"layer": "[a-z0-9_]*"\|"tile_fwd_us": [0-9.]*\|"tile_dgrad_us": [0-9.]*\|"wtile_wgrad_us": [0-9.]*' gpurun_out/b7_layers.log | paste -sd' '
for i in 1 2; do
  step bench 300 python3 bench.py --steps 30 --warmup 5
  echo "bench $(grep -o '"value": [0-9.]*' gpurun_out/b7_bench.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b7_bench.log)"
done
rm -rf gpurun_out/prof_b7
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b7 -o run -- \
  python3 bench.py --steps 5 --warmup 3
python3 scripts/step_breakdown.py gpurun_out/prof_b7/run_kernel_trace.csv --min-us 0 > gpurun_out/step_b7.md 2>&1 || true
tail -2 gpurun_out/step_b7.md
for w in 1 4; do
  step nas_w$w 600 python3 bench/search_throughput.py --candidates 32 --epochs 5 --dataset cifar --graph on \
    --workers-per-device $w
  grep '^{' gpurun_out/b7_nas_w$w.log | cut -c1-400
done
rm -rf gpurun_out/sprof_b7
step nasprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sprof_b7 -o run -- \
  python3 bench/search_throughput.py --candidates 8 --epochs 1 --dataset cifar --graph on
python3 scripts/r4/nas_census.py gpurun_out/sprof_b7 > gpurun_out/b7_nas_census.md 2>&1; head -40 gpurun_out/b7_nas_census.md
