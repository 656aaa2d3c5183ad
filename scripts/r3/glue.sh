#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 scripts/r3/glue_probe.py > gpurun_out/glue_probe.log 2>&1; rc=$?
tail -70 gpurun_out/glue_probe.log; exit $rc
