#!/bin/bash
# fp8 stem: kernel / model tests, then the 128^3 batch-1024 fp8 bench with and without it
# and a kernel trace of the fp8 path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_fp8_stem_gpu.py tests/test_kernels_gpu.py -k "fp8" > gpurun_out/fp8s_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/fp8s_tests.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/fp8s_tests.log | head -20; exit $rc; }
FN_F8_STEM=0 timeout -k 10 300 python3 bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 --steps 3 --warmup 1 --only fp8 > gpurun_out/fp8s_nostem.log 2>&1 || { tail gpurun_out/fp8s_nostem.log; exit 1; }
grep '^{' gpurun_out/fp8s_nostem.log
PROF=1 ACC=0 bash scripts/r3/fp8.sh
