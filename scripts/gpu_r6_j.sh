#!/bin/bash
# Round 6: BN prologue with the loader's transform at raised issue priority; the fixed pipelined
# weight ring; kernel trace.
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
step j_tests 300 python -u -m pytest tests/test_bn_prologue_gpu.py "tests/test_determinism_gpu.py::test_weight_ring_gives_the_register_path_bits" -q -m gpu --timeout 240 --timeout-method thread -p no:cacheprovider || exit $?
FN_BN_PROLOGUE=1 step j_bench_pro 150 python bench.py --steps 30 --warmup 5 || exit $?
FN_BN_PROLOGUE=0 step j_bench_nopro 150 python bench.py --steps 30 --warmup 5 || exit $?
FN_BN_PROLOGUE=0 FN_TILE_WLDS=1 step j_bench_wl 150 python bench.py --steps 30 --warmup 5 || exit $?
R=$GRAFT_REPO_ROOT
cd /tmp && FN_BN_PROLOGUE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/j_prof" -o step -- \
  python3 "$R/bench.py" --steps 5 --warmup 5 > "$R/gpurun_out/j_prof.log" 2>&1
echo "prof rc=$?"
