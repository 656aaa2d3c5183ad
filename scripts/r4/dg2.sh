#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 scripts/r4/dgrad_stats_ab.py > gpurun_out/dg2.log 2>&1; echo "rc=$?"; grep layer gpurun_out/dg2.log
