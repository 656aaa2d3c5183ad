#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_bnfuse_gpu.py > gpurun_out/id3_a.log 2>&1; echo "a rc=$?"
grep -E "passed|failed|rel err|convs.3" gpurun_out/id3_a.log | tail -8
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider "tests/test_bnfuse_gpu.py::test_identity_featurenet3d_matches_colstats" > gpurun_out/id3_b.log 2>&1; echo "b rc=$?"
grep -E "passed|failed|rel err|convs.3" gpurun_out/id3_b.log | tail -8
