#!/bin/bash
# Round 6: the LDS weight ring with the pipelined loader (two DMA batches in flight) against the
# register path, its timing variants (FN_TILE_WLDBG=1: no hand-off waits, 3: no weight DMAs either),
# then the stock PyTorch fp32 oracle (MIOpen find mode, channels-last) on seed 0.
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
  tail -n 2 "gpurun_out/$name.log" | cut -c1-200
  return $rc
}
step f_ring 240 python -u -m pytest "tests/test_determinism_gpu.py::test_weight_ring_gives_the_register_path_bits" -x -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
step f_bench_wl 150 python bench.py --steps 30 --warmup 5 || exit $?
FN_TILE_WLDS=0 step f_bench_reg 150 python bench.py --steps 30 --warmup 5 || exit $?
FN_TILE_WLDBG=1 step f_bench_wl_nowait 150 python bench.py --steps 30 --warmup 5 || exit $?
FN_TILE_WLDBG=3 step f_bench_wl_nodma 150 python bench.py --steps 30 --warmup 5 || exit $?
FN_TILE_WLDS=0 step acc_torch32_s0 700 python -u bench/accuracy.py --impl torch --torch-dtype fp32 --epochs 16 \
  --train-per-class 1000 --seed 0 || exit $?
