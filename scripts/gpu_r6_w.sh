#!/bin/bash
# Round 6: seghead lean instance (no arg-max / logit sum in a training step, exp2 on packed fma,
# full tiles without zero-row selects) and one-instruction bf16 pair packing (conv_tile epilogues):
# the GPU tests that cover them, then the classifier and seg benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_subpixel_gpu.py tests/test_conv_tile_gpu.py tests/test_determinism_gpu.py \
  tests/test_bn_prologue_gpu.py tests/test_bnfuse_gpu.py -q -m gpu --timeout 240 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/w_tests.log 2>&1 || { tail -30 gpurun_out/w_tests.log; exit 1; }
tail -n 1 gpurun_out/w_tests.log
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 30 --warmup 5 > gpurun_out/w_bench_$i.log 2>&1 || exit $?
  tail -n 1 gpurun_out/w_bench_$i.log | cut -c1-150
done
for i in 1 2; do
  timeout -k 10 200 python bench.py --model seg --steps 20 --warmup 5 > gpurun_out/w_seg_$i.log 2>&1 || exit $?
  tail -n 1 gpurun_out/w_seg_$i.log | cut -c1-150
done
