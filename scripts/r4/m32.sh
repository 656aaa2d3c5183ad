#!/bin/bash
# conv_tile32 (32x32x16 MFMA) vs conv_tile (16x16x32): numerics, per-layer times, bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_tile_gpu.py > gpurun_out/m32_pytest.log 2>&1; rc=$?
tail -5 gpurun_out/m32_pytest.log
[ $rc -ne 0 ] && exit $rc
for m in 0 1; do
  FN_TILE_M32=$m timeout -k 10 200 python3 scripts/bench_conv_layers.py --batch 128 --reps 10 > gpurun_out/m32_layers_$m.log 2>&1 || { tail gpurun_out/m32_layers_$m.log; exit 1; }
  grep '^{' gpurun_out/m32_layers_$m.log | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print('m32=$m', r['layer'], 'fwd', r.get('tile_fwd_us'), 'dgrad', r.get('tile_dgrad_us'), r['tile_fwd_plan'][:60])"
done
for m in 1 0 1 0; do
  FN_TILE_M32=$m timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 > gpurun_out/m32_bench_$m.log 2>&1 || { tail gpurun_out/m32_bench_$m.log; exit 1; }
  echo "bench m32=$m $(grep -o '"value": [0-9.]*' gpurun_out/m32_bench_$m.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/m32_bench_$m.log)"
done
