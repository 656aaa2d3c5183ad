#!/bin/bash
# Round-4 batch 6: stem diagnostics (FN_TILE_DBG variants of the space-to-depth stem: cycle stamps,
# no weight loads / no halo reads / no halo DMA), BN-dgrad fusion on the 16x16 kernel A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/b6_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ]; then tail -20 "gpurun_out/b6_$name.log"; exit $rc; fi
  return $rc
}
for d in 0 16 1 2 4; do
  FN_TILE_DBG=$d step stem_$d 120 python -u scripts/bench_conv_layers.py --batch 128 --reps 5 --only stem_s2d
  echo "dbg=$d $(grep -o '"tile_fwd_us": [0-9.]*\|"wtile_wgrad_us": [0-9.]*' gpurun_out/b6_stem_$d.log | tr '\n' ' ') $(grep -o '\[conv_tile stamps.*' gpurun_out/b6_stem_$d.log | head -2 | tr '\n' ' ')"
done
for f in 1 0 1 0; do
  FN_BN_DGRAD_FUSE=$f step bench 300 python3 bench.py --steps 30 --warmup 5
  echo "bench bn_dgrad_fuse=$f $(grep -o '"value": [0-9.]*' gpurun_out/b6_bench.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b6_bench.log)"
done
