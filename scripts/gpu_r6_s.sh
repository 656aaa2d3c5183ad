#!/bin/bash
# Round 6: conv_tile cycle stamps of compute waves 0 and 1 and the loader (experiments build,
# FN_TILE_DBG=16): does wave 0, which shares SIMD 0 with the loader, hold the others at the barrier?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
FN_TILE_DBG=16 timeout -k 10 200 python -u scripts/diag_prologue_stamps.py > gpurun_out/s_stamps.log 2>&1 || exit $?
tail -n 18 gpurun_out/s_stamps.log
