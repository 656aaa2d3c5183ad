#!/bin/bash
# tile-stream multi-pack mismatch diagnosis, the pack tests, benches, seg, step trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python scripts/diag_pack_tile.py > gpurun_out/c13_diag.log 2>&1; echo "diag rc=$?"
grep -v "^/opt" gpurun_out/c13_diag.log | head -40
timeout -k 10 300 python -u -m pytest tests/test_pack_multi_gpu.py -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/c13_tests.log 2>&1; rc=$?
tail -1 gpurun_out/c13_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/c13_tests.log | head
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/c13_bench$i.log 2>&1 || exit $?
  tail -1 gpurun_out/c13_bench$i.log | cut -c1-160
done
timeout -k 10 300 python bench.py --model seg --steps 10 --warmup 3 > gpurun_out/c13_seg.log 2>&1 || exit $?
tail -1 gpurun_out/c13_seg.log | cut -c1-160
