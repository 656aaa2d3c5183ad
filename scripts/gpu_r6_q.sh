#!/bin/bash
# Round 6: schedule counters reused under graph capture (tests that capture the step, benches),
# NAS candidates/hour with a warm 4-worker pool and the kernel census, fp8 inference speed.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_determinism_gpu.py tests/test_rccl_gpu.py tests/test_gpu_pipeline.py tests/test_bnfuse_gpu.py \
  -q -m gpu --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/q_tests.log 2>&1 || { tail -8 gpurun_out/q_tests.log; exit 1; }
tail -n 1 gpurun_out/q_tests.log
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 30 --warmup 5 > gpurun_out/q_bench_$i.log 2>&1 || exit $?
  tail -n 1 gpurun_out/q_bench_$i.log | cut -c1-150
done
timeout -k 10 400 python3 bench/search_throughput.py --candidates 32 --epochs 5 --dataset cifar --graph on \
  --workers-per-device 4 --warm > gpurun_out/q_nas_w4_warm.log 2>&1 || exit $?
echo "nas warm4 $(grep -o '"value": [0-9.]*\|"seconds": [0-9.]*\|"trained": [0-9]*' gpurun_out/q_nas_w4_warm.log | tr '\n' ' ')"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/q_nas_census -o run -- \
  python3 bench/search_throughput.py --candidates 8 --epochs 1 --dataset cifar --graph on > gpurun_out/q_nas_census.log 2>&1 || exit $?
echo "census done"
timeout -k 10 400 python3 bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 > gpurun_out/q_fp8.log 2>&1 || exit $?
tail -n 3 gpurun_out/q_fp8.log | cut -c1-250
