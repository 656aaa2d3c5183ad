#!/bin/bash
# Round 6: the static-only / chunked conv_tile instances and the conv_wtile prologue out of the default
# build -- tests, then the same-box A/B against the round-5 tree (abtest_old/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_determinism_gpu.py tests/test_bn_prologue_gpu.py tests/test_ddp_gpu.py \
  tests/test_rccl_gpu.py tests/test_conv_tile_gpu.py tests/test_conv_wtile_gpu.py -q -m gpu --timeout 240 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/u_tests.log 2>&1 || { tail -8 gpurun_out/u_tests.log; exit 1; }
tail -n 1 gpurun_out/u_tests.log
bash scripts/gpu_ab_tree.sh
