#!/bin/bash
# fp8 inference evaluation on one GPU: the fp8 GPU tests, the 128^3 throughput (block-scaled
# activations vs per-tensor scales, bf16 for reference) and the accuracy parity over 4 seeds.
# Each step has its own time limit; an abort / crash / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n ${TAILN:-6} "gpurun_out/$name.log"
  return $rc
}
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
run fp8_tests 400 python -u -m pytest tests/test_fp8_block_gpu.py tests/test_fp8_stem_gpu.py \
  -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider; rc=$?; if fatal $rc; then exit $rc; fi
run infer_block 300 python bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024; rc=$?; if fatal $rc; then exit $rc; fi
FN_F8_BLOCK=0 run infer_tensor 300 python bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 --only fp8
rc=$?; if fatal $rc; then exit $rc; fi
for s in ${SEEDS:-0 1 2 3}; do
  run acc_seed$s 400 python bench/accuracy.py --fp8 --epochs 16 --train-per-class 1000 --seed $s; rc=$?; if fatal $rc; then exit $rc; fi
done
exit 0
