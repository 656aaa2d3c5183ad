#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_igemm_pack_gpu.py tests/test_determinism_gpu.py tests/test_gpu_pipeline.py tests/test_dense_infer_gpu.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c2_tests.log 2>&1; rc=$?; tail -3 gpurun_out/c2_tests.log; grep -E "FAILED|ERROR" gpurun_out/c2_tests.log | head; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python scripts/diag_nas_step.py --list > gpurun_out/c2_nas.log 2>&1 || exit $?
tail -1 gpurun_out/c2_nas.log
for i in 1 2; do timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/c2_bench$i.log 2>&1 || exit $?; grep -o '"value": [0-9.]*, "unit[^,]*, "n_gpus": 1, "steps": 30, "warmup": 5, "ms_per_step": [0-9.]*' gpurun_out/c2_bench$i.log; done
timeout -k 10 300 python scripts/diag_fp8_parity.py --seed 3 > gpurun_out/c2_parity3.log 2>&1 || exit $?
tail -6 gpurun_out/c2_parity3.log
bash scripts/gpu_tile_budget.sh
