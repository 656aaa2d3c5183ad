#!/bin/bash
# Sub-pixel decoder: BN statistics identity for the encoder's last BN -- tests + seg bench x2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_subpixel_gpu.py tests/test_bnfuse_gpu.py -x -v -m gpu --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/segid_test.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/segid_test.log | tail -1; grep -E "^FAILED|Error" gpurun_out/segid_test.log | head
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --model seg --steps 10 --warmup 3 > gpurun_out/segid_bench.log 2>&1
  rc=$?; echo "seg bench rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/segid_bench.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/segid_bench.log)"
  [ $rc -eq 0 ] || exit $rc
done
FN_BN_IDENTITY=0 timeout -k 10 300 python3 bench.py --model seg --steps 10 --warmup 3 > gpurun_out/segid_bench0.log 2>&1
rc=$?; echo "seg bench (identity off) rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/segid_bench0.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/segid_bench0.log)"
