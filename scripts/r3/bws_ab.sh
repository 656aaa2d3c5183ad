#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_bnfuse_gpu.py tests/test_conv_tile_gpu.py > gpurun_out/bws_tests.log 2>&1
rc=$?; tail -3 gpurun_out/bws_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/bws_tests.log | head; exit $rc; }
for r in 1 2; do for f in 0 1; do
  FN_BN_DGRAD_FUSE=$f timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/bws_$f.log 2>&1 || { tail gpurun_out/bws_$f.log; exit 1; }
  grep '^{' gpurun_out/bws_$f.log | python3 -c "import json,sys; [print('bws $f', (d:=json.loads(l))['value'], d['ms_per_step']) for l in sys.stdin]"
done; done
rm -rf gpurun_out/profbws
FN_BN_DGRAD_FUSE=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/profbws -o run -- \
  python3 bench.py --steps 5 --warmup 3 > gpurun_out/profbws.log 2>&1 || exit 1
python3 scripts/step_breakdown.py gpurun_out/profbws/run_kernel_trace.csv --min-us 40 > gpurun_out/step_bws.md 2>&1; cat gpurun_out/step_bws.md
