#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_subpixel_gpu.py tests/test_bnfuse_gpu.py tests/test_determinism_gpu.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c7_tests.log 2>&1; rc=$?; tail -1 gpurun_out/c7_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/c7_tests.log | head; [ $rc -le 1 ] || exit $rc
for i in 1 2; do timeout -k 10 200 python bench.py --model seg --steps 10 --warmup 3 > gpurun_out/c7_seg$i.log 2>&1 || exit $?; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/c7_seg$i.log | tr '\n' ' '; echo; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c7_nasprof -o run -- python3 bench/search_throughput.py --candidates 8 --epochs 1 --dataset cifar --graph on > gpurun_out/c7_nasprof.log 2>&1 || exit $?
tail -2 gpurun_out/c7_nasprof.log
