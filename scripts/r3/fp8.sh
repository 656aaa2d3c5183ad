#!/bin/bash
# BASELINE config 5: 128^3 fp8 inference at batch 1024 (one 1024-sample forward), kernel trace of the
# tile-F8 path, and trained-model fp8 parity on the tile-F8 kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 --steps 3 --warmup 1 > gpurun_out/r3_fp8_1024.log 2>&1
rc=$?; cat gpurun_out/r3_fp8_1024.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
if [ "${PROF:-1}" = "1" ]; then
  rm -rf gpurun_out/fp8prof
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fp8prof -o run -- \
    python3 bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 --steps 1 --warmup 0 --only ${ONLY:-fp8} > gpurun_out/r3_fp8_prof.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/r3_fp8_prof.log; exit $rc; }
  python3 scripts/prof_summary.py gpurun_out/fp8prof/run_kernel_trace.csv --steps 1 > gpurun_out/r3_fp8_kernels.md 2>&1
  head -30 gpurun_out/r3_fp8_kernels.md
fi
if [ "${ACC:-1}" = "1" ]; then
  timeout -k 10 500 python3 bench/accuracy.py --fp8 --epochs 10 --train-per-class ${TPC:-1000} > gpurun_out/r3_acc_fp8.log 2>&1
  rc=$?; tail -2 gpurun_out/r3_acc_fp8.log | cut -c1-2000; exit $rc
fi
