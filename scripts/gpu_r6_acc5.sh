#!/bin/bash
# Round 6: the bf16-autocast PyTorch oracle on seeds 0-3 and the reference's lenet5-template vs
# hand-written LeNet-5 learning curves (bench/lenet_parity.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_r6_acc3.sh bf16 0 1 2 3 || exit $?
timeout -k 10 300 python -u bench/lenet_parity.py --runs 3 --epochs 12 --report gpurun_out/report_lenet5_parity.txt \
  --out gpurun_out/r6_lenet5_template_vs_handwritten.svg > gpurun_out/lenet_parity.log 2>&1 || exit $?
tail -n 1 gpurun_out/lenet_parity.log | cut -c1-300
