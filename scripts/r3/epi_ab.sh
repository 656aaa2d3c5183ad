#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv_tile_gpu.py tests/test_kernels_gpu.py > gpurun_out/epi_tests.log 2>&1
rc=$?; tail -1 gpurun_out/epi_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/epi_tests.log | head; exit $rc; }
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/epi_b.log 2>&1 || { tail gpurun_out/epi_b.log; exit 1; }
  grep '^{' gpurun_out/epi_b.log | python3 -c "import json,sys; [print('bench', (d:=json.loads(l))['value'], d['ms_per_step']) for l in sys.stdin]"
done
timeout -k 10 150 python3 scripts/bench_conv_layers.py --batch 128 --reps 20 --only stem_s2d,conv2,conv3,conv4 > gpurun_out/epi_layers.log 2>&1 && grep '^{' gpurun_out/epi_layers.log | python3 -c "
import json,sys
for l in sys.stdin: r=json.loads(l); print(r['layer'], 'fwd', r.get('tile_fwd_us'), 'dgrad', r.get('tile_dgrad_us'))"
