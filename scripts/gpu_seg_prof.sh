#!/bin/bash
# Segmentation step kernel trace: rocprofv3 over bench.py --model seg (graph-replayed steps);
# scripts/rocpd_step.py extracts the last step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --model seg --steps 10 --warmup 3 > gpurun_out/sp_seg.log 2>&1 || exit $?
tail -1 gpurun_out/sp_seg.log | cut -c1-200
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/sp_prof" -o seg -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --model seg --steps 3 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/sp_prof.log" 2>&1
echo "prof rc=$?"
