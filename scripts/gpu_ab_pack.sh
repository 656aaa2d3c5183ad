#!/bin/bash
# A/B of the one-launch weight packing (FN_PACK_SCOPE 1 / 0), alternating on one box: training
# bench, seg bench, NAS candidate step; then the pack tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for s in 1 0; do
    FN_PACK_SCOPE=$s timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/abp_cls_$s$r.log 2>&1 || exit $?
    echo "scope=$s cls $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abp_cls_$s$r.log)"
  done
done
for s in 1 0 1 0; do
  FN_PACK_SCOPE=$s timeout -k 10 300 python bench.py --model seg --steps 10 --warmup 3 > gpurun_out/abp_seg_$s.log 2>&1 || exit $?
  echo "scope=$s seg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abp_seg_$s.log)"
done
for s in 1 0 1 0; do
  FN_PACK_SCOPE=$s timeout -k 10 200 python scripts/diag_nas_step.py > gpurun_out/abp_nas_$s.log 2>&1 || exit $?
  echo "scope=$s nas $(tail -1 gpurun_out/abp_nas_$s.log)"
done
timeout -k 10 300 python -u -m pytest tests/test_pack_multi_gpu.py -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/abp_tests.log 2>&1; rc=$?
tail -1 gpurun_out/abp_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/abp_tests.log | head
exit $rc
