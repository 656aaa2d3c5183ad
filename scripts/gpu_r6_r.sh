#!/bin/bash
# Round 6: re-check the weight-gradient / tile-plan defaults against their alternatives on one box
# (alternating benches).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
b() {
  local name=$1; shift
  env "$@" timeout -k 10 150 python bench.py --steps 30 --warmup 5 > gpurun_out/r_$name.log 2>&1 || return $?
  echo "$name $(tail -n 1 gpurun_out/r_$name.log | grep -o '"ms_per_step": [0-9.]*')"
}
b def1 FN_X=0 || exit $?
b nw4 FN_WTILE_NW=4 || exit $?
b ks2off FN_WTILE_KS2=0 || exit $?
b rank1 FN_TILE_PLAN_RANK=1 || exit $?
b rank2 FN_TILE_PLAN_RANK=2 || exit $?
b def2 FN_X=0 || exit $?
b nw4b FN_WTILE_NW=4 || exit $?
b rank1b FN_TILE_PLAN_RANK=1 || exit $?
b def3 FN_X=0 || exit $?
