#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for a in "1 2" "0 2" "0 1"; do
  timeout -k 10 120 python3 scripts/r4/ident_debug3.py $a > gpurun_out/id5.log 2>&1; echo "rc=$?"; grep fork_ident gpurun_out/id5.log
done
