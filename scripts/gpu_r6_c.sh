#!/bin/bash
# Round 6, box 3: the LDS weight ring with a turn-granular hand-off -- bitwise test, bench (ring /
# register path, alternating) and a kernel trace with the ring.
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
step c_ring 240 python -u -m pytest "tests/test_determinism_gpu.py::test_weight_ring_gives_the_register_path_bits" -x -v -s -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
for i in 1 2; do
  step c_bench_wl_$i 150 python bench.py --steps 30 --warmup 5 || exit $?
  FN_TILE_WLDS=0 step c_bench_reg_$i 150 python bench.py --steps 30 --warmup 5 || exit $?
done
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/c_prof_wl" -o step -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/c_prof_wl.log" 2>&1 || exit $?
echo "prof ok"
