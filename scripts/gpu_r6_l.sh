#!/bin/bash
# Round 6: the segmentation head kernel with packed BN / moment math and the 25-class instance
# (tests, bench --model seg, kernel trace), then native seed 3 again on this box (cross-box bits).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 1 "gpurun_out/$name.log" | cut -c1-150
  return $rc
}
step l_tests 400 python -u -m pytest tests/test_subpixel_gpu.py -q -m gpu --timeout 240 --timeout-method thread -p no:cacheprovider || exit $?
step l_seg_1 200 python bench.py --model seg --steps 20 --warmup 5 || exit $?
step l_seg_2 200 python bench.py --model seg --steps 20 --warmup 5 || exit $?
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/l_prof" -o seg -- \
  python3 "$R/bench.py" --model seg --steps 5 --warmup 5 > "$R/gpurun_out/l_prof.log" 2>&1 || exit $?
echo "prof done"
cd "$R" && step acc_native_s3_box2 300 python -u bench/accuracy.py --epochs 16 --train-per-class 1000 --seed 3 --weights-hash
