#!/bin/bash
# Round 6: 64-column workgroups for dgrads into 64 columns (the default now): GPU tests of the
# tile kernel, determinism, BN fusion, sub-pixel and the model kernels, then the benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_conv_tile_gpu.py tests/test_determinism_gpu.py tests/test_bnfuse_gpu.py \
  tests/test_subpixel_gpu.py tests/test_kernels_gpu.py tests/test_ddp_gpu.py tests/test_rccl_gpu.py -q -m gpu --timeout 240 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/af_tests.log 2>&1 || { tail -30 gpurun_out/af_tests.log; exit 1; }
tail -n 1 gpurun_out/af_tests.log
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 30 --warmup 5 > gpurun_out/af_bench_$i.log 2>&1 || exit $?
  tail -n 1 gpurun_out/af_bench_$i.log | cut -c1-140
done
for i in 1 2; do
  timeout -k 10 200 python bench.py --model seg --steps 20 --warmup 5 > gpurun_out/af_seg_$i.log 2>&1 || exit $?
  tail -n 1 gpurun_out/af_seg_$i.log | cut -c1-140
done
