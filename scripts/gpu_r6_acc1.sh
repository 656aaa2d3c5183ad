#!/bin/bash
# Round 6: convergence parity against stock PyTorch (bench/accuracy.py --impl torch) -- the native
# bf16 kernels on 4 seeds (16 epochs, 24k procedural training voxels; weight hashes; seed 3 twice
# in separate processes for the bitwise repeat), then the fp32 PyTorch oracle on seeds 0-1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp FN_TILE_WLDS=${FN_TILE_WLDS:-0}
mkdir -p gpurun_out
for s in 0 1 2 3; do
  timeout -k 10 240 python -u bench/accuracy.py --epochs 16 --train-per-class 1000 --seed $s --weights-hash \
    > gpurun_out/acc_native_s$s.log 2>&1 || exit $?
  tail -n 1 gpurun_out/acc_native_s$s.log | cut -c1-220
done
timeout -k 10 240 python -u bench/accuracy.py --epochs 16 --train-per-class 1000 --seed 3 --weights-hash \
  > gpurun_out/acc_native_s3_repeat.log 2>&1 || exit $?
tail -n 1 gpurun_out/acc_native_s3_repeat.log | cut -c1-220
for s in 0 1; do
  timeout -k 10 420 python -u bench/accuracy.py --impl torch --torch-dtype fp32 --epochs 16 --train-per-class 1000 \
    --seed $s > gpurun_out/acc_torch32_s$s.log 2>&1 || exit $?
  tail -n 1 gpurun_out/acc_torch32_s$s.log | cut -c1-220
done
