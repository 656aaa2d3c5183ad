#!/bin/bash
# fp8 trained-model parity with a second seed; segmentation-head bench on the final tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 bench/accuracy.py --fp8 --epochs 16 --train-per-class 1000 --seed 1 > gpurun_out/r3_acc_fp8_seed1.log 2>&1
rc=$?; tail -1 gpurun_out/r3_acc_fp8_seed1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['fp8'])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model seg --steps 10 --warmup 3 > gpurun_out/r3_bench_seg_final.log 2>&1 || { tail gpurun_out/r3_bench_seg_final.log; exit 1; }
grep '^{' gpurun_out/r3_bench_seg_final.log | cut -c1-200
