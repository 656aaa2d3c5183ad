#!/bin/bash
# Segmentation step (bench.py --model seg): bench x2 + kernel trace of one graph-replayed step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --model seg --steps 10 --warmup 3 > gpurun_out/seg_bench.log 2>&1
  rc=$?; echo "seg bench rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/seg_bench.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/seg_bench.log)"
  [ $rc -eq 0 ] || exit $rc
done
rm -rf gpurun_out/prof_seg
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_seg -o run -- \
  python3 bench.py --model seg --steps 3 --warmup 2 > gpurun_out/seg_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/step_breakdown.py gpurun_out/prof_seg/run_kernel_trace.csv --min-us 0 > gpurun_out/step_seg.md 2>&1
tail -1 gpurun_out/step_seg.md
