#!/bin/bash
# Round 6: kernel traces of the training step with the BN prologue on and off (which kernels the
# prologue slows).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for m in 1 0; do
  cd /tmp && FN_BN_PROLOGUE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/h_prof$m" -o step -- \
    python3 "$R/bench.py" --steps 5 --warmup 5 > "$R/gpurun_out/h_prof$m.log" 2>&1 || exit $?
  echo "prof $m done"
  cd "$R" && python3 scripts/rocpd_step.py $(ls gpurun_out/h_prof$m/*/step_results.db 2>/dev/null | head -1) > gpurun_out/h_step$m.md 2>&1
  tail -2 gpurun_out/h_step$m.md
done
