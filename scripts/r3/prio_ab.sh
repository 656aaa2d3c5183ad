#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv_tile_gpu.py tests/test_fp8_stem_gpu.py > gpurun_out/prio_tests.log 2>&1
rc=$?; tail -1 gpurun_out/prio_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for p in 0 1; do
  FN_TILE_PRIO=$p timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/prio_$p.log 2>&1 || { tail gpurun_out/prio_$p.log; exit 1; }
  grep '^{' gpurun_out/prio_$p.log | python3 -c "import json,sys; [print('prio $p', (d:=json.loads(l))['value'], d['ms_per_step']) for l in sys.stdin]"
done; done
