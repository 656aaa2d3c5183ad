#!/bin/bash
# Stem (8-channel) wgrad variant: tests, per-layer A/B vs the halo wgrad, bench, kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_wtile_gpu.py tests/test_kernels_gpu.py > gpurun_out/c8_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/c8_tests.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/c8_tests.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/bench_conv_layers.py --only stem_s2d > gpurun_out/c8_layers.log 2>&1 || { tail -20 gpurun_out/c8_layers.log; exit 1; }
FN_WTILE_NW=4 timeout -k 10 300 python scripts/bench_conv_layers.py --only stem_s2d > gpurun_out/c8_layers_nw4.log 2>&1 || { tail -20 gpurun_out/c8_layers_nw4.log; exit 1; }
tail -4 gpurun_out/c8_layers.log gpurun_out/c8_layers_nw4.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/c8_bench.log 2>&1 || { tail -20 gpurun_out/c8_bench.log; exit 1; }
grep '^{' gpurun_out/c8_bench.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/c8_prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/c8_prof.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/c8_prof.log"; exit 1; }
