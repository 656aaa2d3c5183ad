#!/bin/bash
# conv_wtile k-step split (FN_WTILE_KS2): wgrad tests, per-layer A/B, bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_wtile_gpu.py > gpurun_out/ks2_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/ks2_tests.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/ks2_tests.log | head -30; exit $rc; }
for v in 1 0; do
FN_WTILE_KS2=$v timeout -k 10 400 python scripts/bench_conv_layers.py --only stem_s2d,conv4,seg_dec > gpurun_out/ks2_layers_$v.log 2>&1 || { tail -20 gpurun_out/ks2_layers_$v.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/ks2_layers_$v.log'):
    if l.startswith('{'):
        r=json.loads(l); print('ks2=$v', r['layer'], {k:v for k,v in r.items() if 'wgrad' in k})
"
done
for v in 1 0; do
  FN_WTILE_KS2=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ks2_bench_$v.log 2>&1 || { tail -20 gpurun_out/ks2_bench_$v.log; exit 1; }
  echo "ks2=$v $(grep '^{' gpurun_out/ks2_bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'])")"
done
