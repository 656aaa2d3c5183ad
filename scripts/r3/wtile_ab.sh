#!/bin/bash
# conv_wtile check: wgrad tests, per-layer timings (LAYERS), bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_wtile_gpu.py > gpurun_out/wab_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/wab_tests.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/wab_tests.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/bench_conv_layers.py --only ${LAYERS:-stem_s2d,conv2,conv3,conv4} > gpurun_out/wab_layers.log 2>&1 || { tail -20 gpurun_out/wab_layers.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/wab_layers.log'):
    if l.startswith('{'):
        r=json.loads(l); print(r['layer'], {k:v for k,v in r.items() if k.endswith('_us')})
"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/wab_bench.log 2>&1 || { tail -20 gpurun_out/wab_bench.log; exit 1; }
grep '^{' gpurun_out/wab_bench.log | python3 -c "import json,sys; [print('bench', (d:=json.loads(l))['value'], d['ms_per_step']) for l in sys.stdin]"
