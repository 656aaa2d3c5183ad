#!/bin/bash
# Round-4 batch 4.  Each step under its own timeout; an ordinary failure (rc 1) is reported and the
# next step runs, a crash / abort / time limit (rc >= 124) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/b4_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ]; then tail -20 "gpurun_out/b4_$name.log"; exit $rc; fi
  return $rc
}
step probe 60 ./scripts/r4/probe/i8_layout; cat gpurun_out/b4_probe.log
step tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_subpixel_gpu.py tests/test_fp8_stem_gpu.py tests/test_bnfuse_gpu.py
grep -E "passed|failed" gpurun_out/b4_tests.log | tail -2; grep -E "^FAILED|Error:" gpurun_out/b4_tests.log | head -10
for x in 1 0 2 1 0; do
  FN_SEG_XENT=$x step seg 300 python3 bench.py --model seg --steps 10 --warmup 3
  echo "seg xent=$x $(grep -o '"value": [0-9.]*' gpurun_out/b4_seg.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b4_seg.log)"
done
for st in 0 i8; do
  FN_F8_STEM=$st step fp8_$st 300 python3 bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024
  echo "fp8 stem=$st"; grep '^{' gpurun_out/b4_fp8_$st.log | cut -c1-300
done
step trial_phases 300 python3 scripts/r4/trial_phases.py --candidates 8 --epochs 5; tail -14 gpurun_out/b4_trial_phases.log
step robust 600 bash scripts/r4/robust.sh; tail -8 gpurun_out/b4_robust.log
step m32pmc 600 bash scripts/r4/m32_pmc.sh; tail -24 gpurun_out/b4_m32pmc.log
