#!/bin/bash
# 128^3 inference with uint8 vs bf16 voxel storage, alternating on one box (block-scaled fp8 and bf16)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in uint8 bf16 uint8 bf16; do
  timeout -k 10 300 python bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 --voxels $v > gpurun_out/iv_$v.log 2>&1 || exit $?
  echo "$v $(grep -o '"precision": "[a-z0-9]*", "value": [0-9.]*\|"ms_per_batch": [0-9.]*' gpurun_out/iv_$v.log | tr '\n' ' ')"
done
