#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
FN_TILE_DBG=16 timeout -k 10 120 python3 scripts/bench_conv_layers.py --batch 128 --reps 1 --only conv2,conv3,conv4 > gpurun_out/tstamps.log 2>&1
rc=$?; grep -v "^{" gpurun_out/tstamps.log | sort | uniq -c | head -40; exit $rc
