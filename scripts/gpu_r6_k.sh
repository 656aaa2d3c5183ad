#!/bin/bash
# Round 6: conv_tile cycle stamps (experiments build, FN_TILE_DBG=16) with the BN prologue on / off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 1 0; do
  FN_TILE_DBG=16 FN_BN_PROLOGUE=$m timeout -k 10 200 python -u scripts/diag_prologue_stamps.py > gpurun_out/k_stamps$m.log 2>&1 || exit $?
  tail -n 12 gpurun_out/k_stamps$m.log
done
