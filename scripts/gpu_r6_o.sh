#!/bin/bash
# Round 6: LeNet-5 template vs hand-written on the hard synthetic set; the seg step after the
# seghead softmax / LDS-constants change (tests, benches, trace).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 240 python -u -m pytest tests/test_subpixel_gpu.py -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/o_tests.log 2>&1 || { tail -5 gpurun_out/o_tests.log; exit 1; }
tail -n 1 gpurun_out/o_tests.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --model seg --steps 20 --warmup 5 > gpurun_out/o_seg_$i.log 2>&1 || exit $?
  tail -n 1 gpurun_out/o_seg_$i.log | cut -c1-160
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/o_prof_seg" -o seg -- \
  python3 "$R/bench.py" --model seg --steps 5 --warmup 5 > "$R/gpurun_out/o_prof_seg.log" 2>&1 || exit $?
cd "$R" && timeout -k 10 400 python -u bench/lenet_parity.py --runs 3 --epochs 12 --hard --report gpurun_out/report_lenet5_parity_hard.txt \
  --out gpurun_out/r6_lenet5_template_vs_handwritten.svg > gpurun_out/lenet_parity_hard.log 2>&1 || exit $?
tail -n 1 gpurun_out/lenet_parity_hard.log | cut -c1-300
