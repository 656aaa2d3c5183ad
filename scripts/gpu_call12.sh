#!/bin/bash
# pack_scope for the tile-kernel streams (FeatureNet-3D / seg encoder): its tests and the suites it
# touches, two training benches, a seg bench, the step's kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_pack_multi_gpu.py tests/test_determinism_gpu.py tests/test_conv_tile_gpu.py \
  tests/test_subpixel_gpu.py tests/test_bnfuse_gpu.py tests/test_kernels_gpu.py -q -m gpu --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/c12_tests.log 2>&1; rc=$?
tail -1 gpurun_out/c12_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/c12_tests.log | head
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/c12_bench$i.log 2>&1 || exit $?
  tail -1 gpurun_out/c12_bench$i.log | cut -c1-160
done
timeout -k 10 300 python bench.py --model seg --steps 10 --warmup 3 > gpurun_out/c12_seg.log 2>&1 || exit $?
tail -1 gpurun_out/c12_seg.log | cut -c1-160
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/c12_prof" -o step -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/c12_prof.log" 2>&1
echo "prof rc=$?"
