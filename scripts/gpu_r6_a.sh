#!/bin/bash
# Round 6: conv_tile after the chunked statistics schedule and the LDS weight ring -- the ring's
# bitwise test first (short limit), then the conv / determinism / RCCL / BN-fusion GPU tests, the
# 1-GPU bench (ring on / off, static schedule; alternating) and the CU-interference sweep
# (scripts/dp_interference.py) of the chunked and the static schedules.  Each GPU step has its own
# time limit; a crash, abort or timeout ends the script.
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
  tail -n 12 "gpurun_out/$name.log"
  return $rc
}
step ring 240 python -u -m pytest "tests/test_determinism_gpu.py::test_weight_ring_gives_the_register_path_bits" -x -v -s -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
for i in 1 2; do
  step bench_wl_$i 150 python bench.py --steps 30 --warmup 5 || exit $?
  FN_TILE_WLDS=0 step bench_reg_$i 150 python bench.py --steps 30 --warmup 5 || exit $?
done
FN_TILE_STATIC=1 FN_TILE_WLDS=0 step bench_r5sched 150 python bench.py --steps 30 --warmup 5 || exit $?
step tests 900 python -u -m pytest tests/test_determinism_gpu.py tests/test_conv_tile_gpu.py tests/test_rccl_gpu.py tests/test_bnfuse_gpu.py tests/test_subpixel_gpu.py -x -v -s -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
step interf_chunk 300 python -u scripts/dp_interference.py --cus 0 8 16 32 --lds 98304 0 --steps 15 || exit $?
FN_TILE_STATIC=1 step interf_static 300 python -u scripts/dp_interference.py --cus 0 8 16 32 --lds 98304 0 --steps 15 || exit $?
