#!/bin/bash
# Round 6: ring bench (once-per-turn count read), the new GPU tests (native Dense dgrad for any K,
# native Dense softmax, the bitwise 2-rank DP test, the RCCL tests), then the first half of the
# convergence-parity runs (scripts/gpu_r6_acc1.sh).
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
step e_ring 240 python -u -m pytest "tests/test_determinism_gpu.py::test_weight_ring_gives_the_register_path_bits" -x -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
for i in 1 2; do
  step e_bench_wl_$i 150 python bench.py --steps 30 --warmup 5 || exit $?
  FN_TILE_WLDS=0 step e_bench_reg_$i 150 python bench.py --steps 30 --warmup 5 || exit $?
done
step e_tests 600 python -u -m pytest tests/test_small_kernels_gpu.py tests/test_ddp_gpu.py tests/test_rccl_gpu.py tests/test_determinism_gpu.py -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
bash scripts/gpu_r6_acc1.sh
