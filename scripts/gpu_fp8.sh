#!/bin/bash
# fp8 inference: kernel numerics tests + 128^3 throughput bench (fp8 vs bf16).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -k "fp8 or segmentation" -p no:cacheprovider \
  > gpurun_out/pytest_fp8.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_fp8.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench/infer_fp8.py --size ${SIZE:-128} --batch ${BATCH:-512} --chunk ${CHUNK:-128} \
  > gpurun_out/infer_fp8.log 2>&1
rc2=$?; tail -4 gpurun_out/infer_fp8.log
exit $rc2
