#!/bin/bash
# Round-4 batch 5: int8 tile-kernel diagnostics, tests of the new paths (bf16-weight dense
# inference, fused pool + BN backward), training bench A/B (FN_POOL_BN_APPLY), fp8 inference
# with the bf16 FC weights, and a step kernel trace.  Each step under its own timeout; a crash /
# abort / time limit (rc >= 124) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/b5_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ]; then tail -20 "gpurun_out/b5_$name.log"; exit $rc; fi
  return $rc
}
step i8dbg 120 python3 scripts/r4/i8_debug.py; cat gpurun_out/b5_i8dbg.log | grep -v amdgpu.ids
step tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_bnfuse_gpu.py "tests/test_kernels_gpu.py::test_dense_infer_bf16_weights" \
  "tests/test_kernels_gpu.py::test_dense_native_matches_fp32" \
  "tests/test_kernels_gpu.py::test_conv_padded_wgrad_cropped_in_kernel" \
  "tests/test_kernels_gpu.py::test_conv_channel_padded" "tests/test_kernels_gpu.py::test_conv_search_space_shapes" \
  "tests/test_kernels_gpu.py::test_conv_fwd_bwd" "tests/test_kernels_gpu.py::test_softmax_xent_dense_bf16" \
  "tests/test_kernels_gpu.py::test_softmax_xent"
grep -E "passed|failed" gpurun_out/b5_tests.log | tail -2; grep -E "^FAILED|Error:" gpurun_out/b5_tests.log | head -10
for a in 1 0 1 0; do
  FN_POOL_BN_APPLY=$a step bench 300 python3 bench.py --steps 30 --warmup 5
  echo "bench pool_bn_apply=$a $(grep -o '"value": [0-9.]*' gpurun_out/b5_bench.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b5_bench.log)"
done
for fc in 1 0; do
  FN_F8_FC_BF16=$fc step fp8_$fc 300 python3 bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024
  echo "fp8 fc_bf16=$fc"; grep '^{' gpurun_out/b5_fp8_$fc.log | cut -c1-300
done
rm -rf gpurun_out/prof_b5
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b5 -o run -- \
  python3 bench.py --steps 5 --warmup 3
python3 scripts/step_breakdown.py gpurun_out/prof_b5/run_kernel_trace.csv --min-us 0 > gpurun_out/step_b5.md 2>&1 || true
tail -3 gpurun_out/step_b5.md
