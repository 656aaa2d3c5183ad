#!/bin/bash
# Round 6: the BN prologue in conv_tile's loader (tests/test_bn_prologue_gpu.py: bitwise against
# bn_apply + conv, model step bitwise) and its bench A/B (register weight path both ways), the LDS
# weight ring with the pipelined loader against the register path, then the stock PyTorch fp32
# oracle (MIOpen find mode, channels-last) on seed 0.
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
step g_pro_tests 300 python -u -m pytest tests/test_bn_prologue_gpu.py "tests/test_determinism_gpu.py::test_weight_ring_gives_the_register_path_bits" -v -m gpu --timeout 240 --timeout-method thread -p no:cacheprovider || exit $?
for i in 1 2; do
  FN_TILE_WLDS=0 FN_BN_PROLOGUE=1 step g_bench_pro_$i 150 python bench.py --steps 30 --warmup 5 || exit $?
  FN_TILE_WLDS=0 FN_BN_PROLOGUE=0 step g_bench_nopro_$i 150 python bench.py --steps 30 --warmup 5 || exit $?
done
FN_TILE_WLDS=1 step g_bench_wl 150 python bench.py --steps 30 --warmup 5 || exit $?
FN_TILE_WLDS=1 FN_TILE_WLDBG=3 step g_bench_wl_nodma 150 python bench.py --steps 30 --warmup 5 || exit $?
FN_TILE_WLDS=0 step acc_torch32_s0 700 python -u bench/accuracy.py --impl torch --torch-dtype fp32 --epochs 16 \
  --train-per-class 1000 --seed 0 || exit $?
