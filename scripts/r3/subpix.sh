#!/bin/bash
# Sub-pixel segmentation decoder: GPU tests, seg bench, step trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_subpixel_gpu.py ${EXTRA_TESTS:-} > gpurun_out/subpix_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/subpix_tests.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/subpix_tests.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --model seg --steps 10 --warmup 3 > gpurun_out/subpix_bench.log 2>&1 || { tail -20 gpurun_out/subpix_bench.log; exit 1; }
grep '^{' gpurun_out/subpix_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('seg', d['value'], d['ms_per_step'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/subpix_prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --model seg --steps 3 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/subpix_prof.log" 2>&1 || exit 1
