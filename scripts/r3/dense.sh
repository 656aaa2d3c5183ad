#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py tests/test_small_kernels_gpu.py -k "dense or linear or fc" > gpurun_out/dense_tests.log 2>&1
rc=$?; tail -2 gpurun_out/dense_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/dense_tests.log | head; exit $rc; }
timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/dense_bench.log 2>&1 || { tail gpurun_out/dense_bench.log; exit 1; }
grep '^{' gpurun_out/dense_bench.log | python3 -c "import json,sys; [print('bench', (d:=json.loads(l))['value'], d['ms_per_step']) for l in sys.stdin]"
PROF=1 ACC=0 bash scripts/r3/fp8.sh > /dev/null 2>&1; grep -v amdgpu gpurun_out/r3_fp8_1024.log
grep -i "dense" gpurun_out/r3_fp8_kernels.md | head -4
