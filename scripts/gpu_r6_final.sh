#!/bin/bash
# Round 6, end: the whole GPU suite and smoke() (part 1), or the benches and kernel traces (part 2).
#   bash scripts/gpu_r6_final.sh suite | bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
if [ "$1" = suite ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/final_pytest_gpu.log 2>&1
  rc=$?
  tail -n 3 gpurun_out/final_pytest_gpu.log; grep -E "^FAILED|^ERROR" gpurun_out/final_pytest_gpu.log | head -20
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || exit $?
  tail -n 1 gpurun_out/final_smoke.log
  exit 0
fi
timeout -k 10 300 python -u -m pytest tests/test_subpixel_gpu.py -q -m gpu --timeout 200 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/final_subpixel.log 2>&1 || { tail -5 gpurun_out/final_subpixel.log; exit 1; }
tail -n 1 gpurun_out/final_subpixel.log
for i in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 30 --warmup 5 > gpurun_out/final_bench_$i.log 2>&1 || exit $?
  tail -n 1 gpurun_out/final_bench_$i.log | cut -c1-160
done
for i in 1 2; do
  timeout -k 10 200 python bench.py --model seg --steps 20 --warmup 5 > gpurun_out/final_seg_$i.log 2>&1 || exit $?
  tail -n 1 gpurun_out/final_seg_$i.log | cut -c1-160
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/final_prof" -o step -- \
  python3 "$R/bench.py" --steps 5 --warmup 5 > "$R/gpurun_out/final_prof.log" 2>&1 || exit $?
echo "prof done"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/final_prof_seg" -o seg -- \
  python3 "$R/bench.py" --model seg --steps 5 --warmup 5 > "$R/gpurun_out/final_prof_seg.log" 2>&1 || exit $?
echo "prof seg done"
