#!/bin/bash
# Round 6: NAS candidates/hour against the worker count (warm pools, 64 CIFAR LeNet mutants x 5
# epochs, hipGraph steps): the best worker count for the 20K/h target.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
# (and the measured per-parameter errors of the composed FeatureNet-3D test, to set its bounds)
timeout -k 10 200 python -u -m pytest "tests/test_kernels_gpu.py::test_featurenet3d_matches_reference_step" -s -q -m gpu \
  --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/v_compose.log 2>&1 || { tail -20 gpurun_out/v_compose.log; exit 1; }
grep -c "rel=" gpurun_out/v_compose.log
for w in ${NAS_WORKERS:-3 4 5 6 8}; do
  timeout -k 10 400 python3 bench/search_throughput.py --candidates 64 --epochs 5 --dataset cifar --graph on \
    --workers-per-device $w --warm > gpurun_out/v_nas_w${w}.log 2>&1 || exit $?
  echo "nas warm$w $(grep -o '"value": [0-9.]*\|"seconds": [0-9.]*\|"trained": [0-9]*' gpurun_out/v_nas_w${w}.log | tr '\n' ' ')"
done
