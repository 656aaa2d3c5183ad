#!/bin/bash
# GPU test suite, 1-GPU bench twice, fp8 inference speed (block / per-tensor) and the 4-seed
# fp8 parity (1000 samples/class x 16 epochs).  Each step under its own time limit; a crash or
# timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n ${TAILN:-3} "gpurun_out/$name.log" | cut -c1-400
  return $rc
}
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  run r_pytest 1000 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
  rc=$?; if fatal $rc; then exit $rc; fi
  grep -E "FAILED|ERROR" gpurun_out/r_pytest.log | head -20
fi
for i in 1 2; do run r_bench$i 200 python bench.py --steps 30 --warmup 5 || exit $?; done
run r_infer_block 300 python bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 || exit $?
FN_F8_BLOCK=0 run r_infer_tensor 300 python bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 --only fp8 || exit $?
for s in ${SEEDS:-0 1 2 3}; do
  run r_acc$s 400 python bench/accuracy.py --fp8 --epochs 16 --train-per-class 1000 --seed $s; rc=$?
  if fatal $rc; then exit $rc; fi
done
exit 0
