#!/bin/bash
# A/B of conv_tile's 8-compute-wave form (FN_TILE_W8): per-layer kernel times (bench_conv_layers)
# and whole training / segmentation steps, alternating on one box.  W8S: the FN_TILE_W8 values
# (1 = everywhere it fits, -1 = never, 0 = the default rule).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
W8S=${W8S:-0 1 0 1}
for w in $W8S; do
  FN_TILE_W8=$w timeout -k 10 200 python -u scripts/bench_conv_layers.py --batch 128 --reps 5 --tile-only \
    > gpurun_out/w8_layers_$w.log 2>&1 || exit $?
  echo "w8=$w $(grep -o '"layer": "[a-z0-9_]*"\|"tile_[a-z_]*_us": [0-9.]*' gpurun_out/w8_layers_$w.log | tr '\n' ' ')"
done
for w in $W8S; do
  FN_TILE_W8=$w timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/w8_cls_$w.log 2>&1 || exit $?
  echo "cls w8=$w $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/w8_cls_$w.log)"
  FN_TILE_W8=$w timeout -k 10 200 python bench.py --model seg --steps 10 --warmup 3 > gpurun_out/w8_seg_$w.log 2>&1 || exit $?
  echo "seg w8=$w $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/w8_seg_$w.log)"
done
FN_TILE_W8=1 timeout -k 10 300 python -u -m pytest tests/test_conv_tile_gpu.py tests/test_determinism_gpu.py -q -m gpu \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/w8_tests.log 2>&1; rc=$?
tail -1 gpurun_out/w8_tests.log; exit $rc
