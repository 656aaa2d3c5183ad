#!/bin/bash
# fp8 / bf16 inference at 128^3 with uint8 voxels: the numerics tests, then the speed bench
# (block-scaled default, then per-tensor)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fp8_block_gpu.py tests/test_fp8_stem_gpu.py tests/test_u8_input_gpu.py -q -m gpu \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/iu_tests.log 2>&1; rc=$?
tail -1 gpurun_out/iu_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/iu_tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 > gpurun_out/iu_block.log 2>&1 || exit $?
grep '"value"\|speedup' gpurun_out/iu_block.log | cut -c1-250
FN_F8_BLOCK=0 timeout -k 10 300 python bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 --only fp8 > gpurun_out/iu_tensor.log 2>&1 || exit $?
grep '"value"' gpurun_out/iu_tensor.log | cut -c1-250
