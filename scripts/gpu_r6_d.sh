#!/bin/bash
# Round 6, box 4: where the LDS weight ring loses (the ring without its hand-off, timing only), and
# the burst-interference sweep of the static and the chunked BN-statistics schedules.
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
FN_TILE_WLDBG=1 step d_bench_nowait 150 python bench.py --steps 30 --warmup 5 || exit $?
step d_bench_wl 150 python bench.py --steps 30 --warmup 5 || exit $?
FN_TILE_WLDS=0 step d_bench_reg 150 python bench.py --steps 30 --warmup 5 || exit $?
cd /tmp
FN_TILE_WLDBG=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/d_prof_nowait" -o step -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/d_prof_nowait.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
FN_TILE_WLDS=0 step d_interf 500 python -u scripts/dp_interference.py --cus 8 16 32 --lds 98304 0 --burst-us 300 --offsets 8 --reps 6 || exit $?
