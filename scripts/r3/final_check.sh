#!/bin/bash
# Round-end style check: GPU suite, smoke, bench (N=1), kernel-trace profile of the step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SKIP_TORCH=1 STEPS=30 bash scripts/gpu_check.sh || exit $?
rm -rf gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 bench.py --steps 5 --warmup 3 > gpurun_out/prof_bench.log 2>&1 || { tail -5 gpurun_out/prof_bench.log; exit 1; }
python3 scripts/step_breakdown.py gpurun_out/prof/run_kernel_trace.csv --min-us 0 > gpurun_out/step_breakdown.md 2>&1 || true
tail -5 gpurun_out/step_breakdown.md
