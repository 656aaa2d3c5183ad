#!/bin/bash
# Round 6: 64-column conv_tile workgroups (MT 4 x NT 4) for the classifier's 64-column convs
# (FN_TILE_NT4=1): the tile-kernel GPU tests under it, then the bench alternating 1 / 0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
FN_TILE_NT4=1 timeout -k 10 500 python -u -m pytest tests/test_conv_tile_gpu.py tests/test_determinism_gpu.py tests/test_bnfuse_gpu.py \
  -q -m gpu --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/ad_tests.log 2>&1 || { tail -30 gpurun_out/ad_tests.log; exit 1; }
tail -n 1 gpurun_out/ad_tests.log
for i in 1 2; do
  for f in 1 0; do
    FN_TILE_NT4=$f timeout -k 10 150 python bench.py --steps 30 --warmup 5 > gpurun_out/ad_bench_${f}_$i.log 2>&1 || exit $?
    echo "nt4=$f $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/ad_bench_${f}_$i.log | tr '\n' ' ')"
  done
done
