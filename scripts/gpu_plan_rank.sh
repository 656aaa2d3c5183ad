#!/bin/bash
# conv_tile planner check: per-layer forward / dgrad / masked-dgrad times of the k-th cheapest plan
# (FN_TILE_PLAN_RANK = 0 .. 3, then 0 again), FeatureNet-3D shapes at batch 128
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 0 1 2 3 0; do
  FN_TILE_PLAN_RANK=$k timeout -k 10 200 python -u scripts/bench_conv_layers.py --batch 128 --reps 5 --tile-only \
    > gpurun_out/rank_$k.log 2>&1 || exit $?
  echo "rank=$k $(grep -o '"layer": "[a-z0-9_]*"\|"tile_[a-z_]*_us": [0-9.]*\|"tile_[a-z_]*plan": "TilePlan(TD=[0-9]*, TH=[0-9]*, TW=[0-9]*' gpurun_out/rank_$k.log | tr '\n' ' ')"
done
