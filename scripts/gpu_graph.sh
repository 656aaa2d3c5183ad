#!/bin/bash
# hipGraph training-step test + NAS search throughput (graph vs eager).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -s -k "graph or fp8 or space_to_depth" \
  -p no:cacheprovider > gpurun_out/pytest_graph.log 2>&1
rc=$?; grep -E "step time|passed|failed" gpurun_out/pytest_graph.log | tail -4
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench/search_throughput.py --candidates ${CANDS:-8} > gpurun_out/search_throughput.log 2>&1
rc2=$?; tail -3 gpurun_out/search_throughput.log
exit $rc2
