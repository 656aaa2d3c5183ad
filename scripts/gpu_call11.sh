#!/bin/bash
# one-launch weight packing (pack_scope): its tests, the gather / halo / NAS tests it touches,
# the NAS step kernel list, FC A/B after the dgrad / wgrad revert, a training bench and the NAS
# throughput at 1 and 4 workers
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_pack_multi_gpu.py tests/test_igemm_pack_gpu.py tests/test_determinism_gpu.py \
  tests/test_gpu_pipeline.py tests/test_kernels_gpu.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/c11_tests.log 2>&1; rc=$?
tail -1 gpurun_out/c11_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/c11_tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/diag_nas_step.py --list --stacks > gpurun_out/c11_nas_stacks.log 2>&1 || exit $?
tail -1 gpurun_out/c11_nas_stacks.log
timeout -k 10 120 python scripts/bench_fc_native.py --batch 128 --reps 50 > gpurun_out/c11_fc.log 2>&1 || exit $?
echo "fc $(tail -1 gpurun_out/c11_fc.log)"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/c11_bench.log 2>&1 || exit $?
tail -1 gpurun_out/c11_bench.log | cut -c1-200
WORKERS="1 4" timeout -k 10 700 bash scripts/gpu_nas.sh 2>&1 | grep -v "^$" | head -5
