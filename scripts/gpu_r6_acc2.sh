#!/bin/bash
# Round 6: the fp32 PyTorch oracle on seeds 2-3, the bf16-autocast PyTorch run on seeds 0-3, and the
# reference's lenet5-template vs hand-written LeNet-5 learning curves (bench/lenet_parity.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp FN_TILE_WLDS=${FN_TILE_WLDS:-0}
mkdir -p gpurun_out
for s in 2 3; do
  timeout -k 10 420 python -u bench/accuracy.py --impl torch --torch-dtype fp32 --epochs 16 --train-per-class 1000 \
    --seed $s > gpurun_out/acc_torch32_s$s.log 2>&1 || exit $?
  tail -n 1 gpurun_out/acc_torch32_s$s.log | cut -c1-220
done
for s in 0 1 2 3; do
  timeout -k 10 300 python -u bench/accuracy.py --impl torch --torch-dtype bf16 --epochs 16 --train-per-class 1000 \
    --seed $s > gpurun_out/acc_torch16_s$s.log 2>&1 || exit $?
  tail -n 1 gpurun_out/acc_torch16_s$s.log | cut -c1-220
done
timeout -k 10 300 python -u bench/lenet_parity.py --runs 3 --epochs 12 --report gpurun_out/report_lenet5_parity.txt \
  --out gpurun_out/r6_lenet5_template_vs_handwritten.svg > gpurun_out/lenet_parity.log 2>&1 || exit $?
tail -n 1 gpurun_out/lenet_parity.log | cut -c1-300
