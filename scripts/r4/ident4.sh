#!/bin/bash
# bisect: which earlier test makes FeatureNet-3D's conv4 weight gradient differ run to run
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=tests/test_bnfuse_gpu.py
run() {
  local name=$1; shift
  timeout -k 10 200 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread -p no:cacheprovider "$@" \
    "$T::test_identity_featurenet3d_matches_colstats" > gpurun_out/id4_$name.log 2>&1
  echo "$name rc=$? $(grep -o "convs.3.weight': '[^']*'" gpurun_out/id4_$name.log | head -1)"
}
run pool "$T::test_pool_bwd_bn_stats_match_colstats"
run apply "$T::test_pool_bn_bwd_apply_matches_separate_passes"
run seg "$T::test_seg_head_bn_in_pointwise_matches_unfused"
run fork "$T::test_forked_bn_output_falls_back"
