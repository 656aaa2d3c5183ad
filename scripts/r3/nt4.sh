#!/bin/bash
# 64-column conv_tile workgroups (NT = 4): numerics tests, per-layer A/B vs NT = 2, bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv_tile_gpu.py tests/test_subpixel_gpu.py > gpurun_out/nt4_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/nt4_tests.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/nt4_tests.log | head -20; exit $rc; }
for nt in 2 auto; do
  FN_TILE_NT=$nt timeout -k 10 300 python scripts/bench_conv_layers.py --reps 20 --only conv3,conv4 > gpurun_out/nt4_layers_$nt.log 2>&1 || { tail -20 gpurun_out/nt4_layers_$nt.log; exit 1; }
  python3 -c "
import json,sys
for l in open('gpurun_out/nt4_layers_$nt.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$nt', d['layer'], 'fwd', d.get('tile_fwd_us'), 'dgrad', d.get('tile_dgrad_us'))"
done
for nt in 2 auto; do
  FN_TILE_NT=$nt timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/nt4_bench_$nt.log 2>&1 || { tail -20 gpurun_out/nt4_bench_$nt.log; exit 1; }
  grep '^{' gpurun_out/nt4_bench_$nt.log | python3 -c "import json,sys; [print('bench $nt', (d:=json.loads(l))['value'], d['ms_per_step']) for l in sys.stdin]"
done
