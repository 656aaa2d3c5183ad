#!/bin/bash
# Robustness evaluation seconds per candidate (CW + PGD + CLEVER on the 500-sample set,
# bench/robustness.py defaults).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench/robustness.py > gpurun_out/robustness.log 2>&1 || exit $?
tail -1 gpurun_out/robustness.log | cut -c1-400
