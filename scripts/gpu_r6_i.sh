#!/bin/bash
# Round 6: the BN prologue after the packed-transform rewrite -- tests, bench A/B (z written by the
# forward loader / normalised again by the weight gradients / bn_apply), a kernel trace.
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
step i_tests 300 python -u -m pytest tests/test_bn_prologue_gpu.py -q -m gpu --timeout 240 --timeout-method thread -p no:cacheprovider || exit $?
for i in 1 2; do
  FN_BN_PROLOGUE=1 step i_bench_pro_$i 150 python bench.py --steps 30 --warmup 5 || exit $?
  FN_BN_PROLOGUE=1 FN_BN_PROLOGUE_WGRAD=1 step i_bench_prow_$i 150 python bench.py --steps 30 --warmup 5 || exit $?
  FN_BN_PROLOGUE=0 step i_bench_nopro_$i 150 python bench.py --steps 30 --warmup 5 || exit $?
done
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/i_prof" -o step -- \
  python3 "$R/bench.py" --steps 5 --warmup 5 > "$R/gpurun_out/i_prof.log" 2>&1
echo "prof rc=$?"
