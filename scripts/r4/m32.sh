#!/bin/bash
# conv_tile32 (32x32x16 MFMA) vs conv_tile (16x16x32): numerics, per-layer times, bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_tile_gpu.py tests/test_bnfuse_gpu.py > gpurun_out/m32_pytest.log 2>&1; rc=$?
tail -5 gpurun_out/m32_pytest.log
[ $rc -ne 0 ] && exit $rc
for m in 0 1; do
  FN_TILE_M32=$m timeout -k 10 200 python3 scripts/bench_conv_layers.py --batch 128 --reps 10 > gpurun_out/m32_layers_$m.log 2>&1 || { tail gpurun_out/m32_layers_$m.log; exit 1; }
  grep '^{' gpurun_out/m32_layers_$m.log | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print('m32=$m', r['layer'], 'fwd', r.get('tile_fwd_us'), 'dgrad', r.get('tile_dgrad_us'), r['tile_fwd_plan'][:60])"
done
# m32 on / off, and m32 without the dgrad-epilogue BN statistics
for cfg in "1 auto" "0 auto" "1 0" "1 auto" "0 auto" "1 0"; do
  set -- $cfg
  FN_TILE_M32=$1 FN_BN_DGRAD_FUSE=$2 timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 > gpurun_out/m32_bench.log 2>&1 || { tail gpurun_out/m32_bench.log; exit 1; }
  echo "bench m32=$1 bnfuse=$2 $(grep -o '"value": [0-9.]*' gpurun_out/m32_bench.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/m32_bench.log)"
done
rm -rf gpurun_out/prof_m32
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_m32 -o run -- \
  python3 bench.py --steps 5 --warmup 3 > gpurun_out/prof_m32_bench.log 2>&1 || { tail -5 gpurun_out/prof_m32_bench.log; exit 1; }
python3 scripts/step_breakdown.py gpurun_out/prof_m32/run_kernel_trace.csv --min-us 0 > gpurun_out/step_m32.md 2>&1 || true
tail -40 gpurun_out/step_m32.md
