#!/bin/bash
# Round 6: the calibration-driven fp8 fallback (quantize_model(fallback=True)): its GPU test, then
# trained models (16 epochs, seeds given) evaluated in fp8 with every scale form and the fallback.
#   bash scripts/gpu_r6_y.sh 0 1 2 3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fp8_block_gpu.py tests/test_fp8_stem_gpu.py -q -m gpu --timeout 240 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/y_tests.log 2>&1 || { tail -30 gpurun_out/y_tests.log; exit 1; }
tail -n 1 gpurun_out/y_tests.log
for s in "$@"; do
  timeout -k 10 400 python -u bench/accuracy.py --fp8 --epochs 16 --train-per-class 1000 --seed $s \
    > gpurun_out/y_acc_s$s.log 2>&1 || exit $?
  tail -n 1 gpurun_out/y_acc_s$s.log | grep -o '"top1_bf16": [0-9.]*\|"auto_fallback": {[^}]*}' | tr '\n' ' '; echo
done
