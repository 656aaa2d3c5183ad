#!/bin/bash
# rocprofv3 kernel stats of the 128^3 fp8 inference, block-scaled and per-tensor activations.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for mode in 1 0; do
  FN_F8_BLOCK=$mode timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f8_$mode -o run -- \
    python bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 --only fp8 --steps 1 --warmup 1 \
    > gpurun_out/prof_f8_$mode.log 2>&1 || exit $?
  tail -2 gpurun_out/prof_f8_$mode.log
done
