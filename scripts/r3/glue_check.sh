#!/bin/bash
# GPU suite, then the NAS glue census and throughput after the glue removal.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 400 python3 scripts/r3/glue_probe.py > gpurun_out/glue_probe.log 2>&1 || { tail -20 gpurun_out/glue_probe.log; exit 1; }
tail -30 gpurun_out/glue_probe.log
bash scripts/r3/nas.sh
