#!/bin/bash
# Round 6, box 2: the LDS weight ring with the pipelined loader and the XCD-queue chunk schedule --
# the ring's bitwise test, the bench (ring / register path / round-5 static schedule, alternating)
# and a kernel trace of each schedule (register path).  Each GPU step has its own time limit.
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
  tail -n 3 "gpurun_out/$name.log" | cut -c1-300
  return $rc
}
step b_ring 240 python -u -m pytest "tests/test_determinism_gpu.py::test_weight_ring_gives_the_register_path_bits" "tests/test_determinism_gpu.py::test_tile_statistics_do_not_depend_on_the_grid" -x -v -s -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
for i in 1 2; do
  step b_bench_wl_$i 150 python bench.py --steps 30 --warmup 5 || exit $?
  FN_TILE_WLDS=0 step b_bench_reg_$i 150 python bench.py --steps 30 --warmup 5 || exit $?
  FN_TILE_STATIC=1 FN_TILE_WLDS=0 step b_bench_static_$i 150 python bench.py --steps 30 --warmup 5 || exit $?
done
cd /tmp
for v in reg static wl; do
  case $v in reg) export FN_TILE_WLDS=0 FN_TILE_STATIC=0;; static) export FN_TILE_WLDS=0 FN_TILE_STATIC=1;; wl) export FN_TILE_WLDS=1 FN_TILE_STATIC=0;; esac
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/b_prof_$v" -o step -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/b_prof_$v.log" 2>&1 || exit $?
  echo "prof $v ok"
done
