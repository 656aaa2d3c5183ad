#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_fp8_stem_gpu.py > gpurun_out/f8diag.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/f8diag.log | tail -2; grep -E "FAILED|Error|assert|same" gpurun_out/f8diag.log | head -20; exit $rc
