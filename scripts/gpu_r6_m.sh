#!/bin/bash
# Round 6: the row form of the shifted-layout BN backward (seg) and compile-time activations in the
# pool / BN-pool passes: tests, bench --model seg and the classifier bench, traces.
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
step m_tests 500 python -u -m pytest tests/test_subpixel_gpu.py tests/test_determinism_gpu.py tests/test_kernels_gpu.py -q -m gpu --timeout 240 --timeout-method thread -p no:cacheprovider || exit $?
step m_seg_1 200 python bench.py --model seg --steps 20 --warmup 5 || exit $?
step m_seg_2 200 python bench.py --model seg --steps 20 --warmup 5 || exit $?
step m_bench_1 150 python bench.py --steps 30 --warmup 5 || exit $?
step m_bench_2 150 python bench.py --steps 30 --warmup 5 || exit $?
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/m_prof" -o seg -- \
  python3 "$R/bench.py" --model seg --steps 5 --warmup 5 > "$R/gpurun_out/m_prof.log" 2>&1
echo "prof rc=$?"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/m_prof_cls" -o step -- \
  python3 "$R/bench.py" --steps 5 --warmup 5 > "$R/gpurun_out/m_prof_cls.log" 2>&1
echo "prof cls rc=$?"
