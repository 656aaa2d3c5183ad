#!/bin/bash
# Round 6: the sub-pixel dgrad on 64-column workgroups (conv_tile MT 4 x NT 4): its GPU tests,
# then the seg bench alternating FN_SUBPIXEL_NT4=1 / 0 on one box, and a seg kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_subpixel_gpu.py tests/test_conv_tile_gpu.py -q -m gpu --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/ac_tests.log 2>&1 || { tail -30 gpurun_out/ac_tests.log; exit 1; }
tail -n 1 gpurun_out/ac_tests.log
for i in 1 2; do
  for f in 1 0; do
    FN_SUBPIXEL_NT4=$f timeout -k 10 200 python bench.py --model seg --steps 20 --warmup 5 > gpurun_out/ac_seg_${f}_$i.log 2>&1 || exit $?
    echo "nt4=$f $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/ac_seg_${f}_$i.log | tr '\n' ' ')"
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/ac_prof" -o seg -- \
  python3 "$R/bench.py" --model seg --steps 5 --warmup 5 > "$R/gpurun_out/ac_prof.log" 2>&1 || exit $?
echo "prof done"
