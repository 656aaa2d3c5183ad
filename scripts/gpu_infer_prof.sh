#!/bin/bash
# 128^3 inference (bf16 and fp8) under rocprofv3 --kernel-trace --stats, plus the
# trained-model fp8 parity run of bench/accuracy.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/iprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/iprof -o run -- \
  python3 bench/infer_fp8.py --size 128 --batch 256 --chunk 128 --steps 1 --warmup 1 > gpurun_out/iprof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/iprof.log
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/iprof -name "*kernel_stats.csv" | head -1); head -30 "$f"
timeout -k 10 400 python3 bench/accuracy.py --train-per-class ${TPC:-1000} --epochs 10 --fp8 > gpurun_out/acc_fp8.log 2>&1
rc=$?; tail -1 gpurun_out/acc_fp8.log; exit $rc
