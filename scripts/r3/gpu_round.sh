#!/bin/bash
# Round-3 GPU check: selected tests (TESTS), conv_tile constant-offset experiment, bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider $TESTS > gpurun_out/r3_tests.log 2>&1
  rc=$?; grep -E "passed|failed|error" gpurun_out/r3_tests.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r3_tests.log | head -20; exit $rc; }
fi
if [ "${EXP:-0}" = "1" ]; then bash scripts/r3/tile_dbg2.sh || exit 1; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench.log 2>&1 || { tail -20 gpurun_out/r3_bench.log; exit 1; }
grep '^{' gpurun_out/r3_bench.log | python3 -c "import json,sys; [print('bench', (d:=json.loads(l))['value'], d['ms_per_step'], d.get('graph_fallback')) for l in sys.stdin]"
