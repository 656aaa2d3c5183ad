#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 scripts/r4/ident_debug2.py > gpurun_out/id2_debug.log 2>&1; echo "rc=$?"; grep -v amdgpu.ids gpurun_out/id2_debug.log | tail -30
