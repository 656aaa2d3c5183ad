#!/bin/bash
# Round-4 (session 2): full GPU suite, smoke, fp8 inference A/B, fp8 parity (2 seeds), seg bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/f1_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ]; then tail -20 "gpurun_out/f1_$name.log"; exit $rc; fi
  return $rc
}
step tests 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
grep -E "passed|failed" gpurun_out/f1_tests.log | tail -2; grep -E "^FAILED" gpurun_out/f1_tests.log | head -5
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; tail -1 gpurun_out/f1_smoke.log
step fp8 300 python3 bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024
grep '^{' gpurun_out/f1_fp8.log | cut -c1-220
for seed in 0 1; do
  step acc_$seed 600 python3 bench/accuracy.py --epochs 16 --train-per-class 1000 --fp8 --seed $seed
  grep -o '"top1_bf16": [0-9.]*, "top1_fp8": [0-9.]*, "drop_pt": [-0-9.]*, "agreement": [0-9.]*' gpurun_out/f1_acc_$seed.log | head -1
done
step seg 300 python3 bench.py --model seg --steps 10 --warmup 3
echo "seg $(grep -o '"value": [0-9.]*' gpurun_out/f1_seg.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/f1_seg.log)"
