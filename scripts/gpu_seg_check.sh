#!/bin/bash
# After a change on the segmentation path: its GPU tests, two seg benches and the seg step trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_subpixel_gpu.py tests/test_determinism_gpu.py tests/test_bnfuse_gpu.py \
  tests/test_u8_input_gpu.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/sc_tests.log 2>&1; rc=$?
tail -1 gpurun_out/sc_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/sc_tests.log | head
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --model seg --steps 10 --warmup 3 > gpurun_out/sc_seg$i.log 2>&1 || exit $?
  tail -1 gpurun_out/sc_seg$i.log | cut -c1-160
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/sc_prof" -o seg -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --model seg --steps 3 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/sc_prof.log" 2>&1
echo "prof rc=$?"
