#!/bin/bash
# Round-4 batch 8: the int8 stem after the epilogue fix (tests, inference A/B, trained-model parity
# on two seeds), the training bench + step trace after the dense / NAS fixes, NAS throughput.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/b8_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ]; then tail -20 "gpurun_out/b8_$name.log"; exit $rc; fi
  return $rc
}
step i8dbg 120 python3 scripts/r4/i8_debug.py; grep -v amdgpu.ids gpurun_out/b8_i8dbg.log | tail -6
step tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_fp8_stem_gpu.py "tests/test_kernels_gpu.py::test_dense_native_matches_fp32" \
  "tests/test_kernels_gpu.py::test_conv_padded_wgrad_cropped_in_kernel" "tests/test_kernels_gpu.py::test_conv_channel_padded" \
  "tests/test_kernels_gpu.py::test_conv_search_space_shapes"
grep -E "passed|failed" gpurun_out/b8_tests.log | tail -2; grep -E "^FAILED|Error:" gpurun_out/b8_tests.log | head -10
for st in i8 0; do
  FN_F8_STEM=$st step fp8_$st 300 python3 bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024
  echo "fp8 stem=$st"; grep '^{' gpurun_out/b8_fp8_$st.log | cut -c1-300
done
for seed in 0 1; do
  step acc_$seed 600 python3 bench/accuracy.py --epochs 16 --train-per-class 1000 --fp8 --seed $seed
  grep -o '"fp8": {.*' gpurun_out/b8_acc_$seed.log | cut -c1-600
done
for i in 1 2; do
  step bench 300 python3 bench.py --steps 30 --warmup 5
  echo "bench $(grep -o '"value": [0-9.]*' gpurun_out/b8_bench.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b8_bench.log)"
done
rm -rf gpurun_out/prof_b8
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b8 -o run -- \
  python3 bench.py --steps 5 --warmup 3
python3 scripts/step_breakdown.py gpurun_out/prof_b8/run_kernel_trace.csv --min-us 0 > gpurun_out/step_b8.md 2>&1 || true
tail -2 gpurun_out/step_b8.md
