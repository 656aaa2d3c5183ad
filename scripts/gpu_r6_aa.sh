#!/bin/bash
# Round 6: the shifted-layout BN backward with one pass per row (5 / 8 chunks per thread): the
# sub-pixel GPU tests, the seg bench and a seg kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_subpixel_gpu.py -q -m gpu --timeout 200 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/aa_tests.log 2>&1 || { tail -30 gpurun_out/aa_tests.log; exit 1; }
tail -n 1 gpurun_out/aa_tests.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --model seg --steps 20 --warmup 5 > gpurun_out/aa_seg_$i.log 2>&1 || exit $?
  tail -n 1 gpurun_out/aa_seg_$i.log | cut -c1-140
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/aa_prof" -o seg -- \
  python3 "$R/bench.py" --model seg --steps 5 --warmup 5 > "$R/gpurun_out/aa_prof.log" 2>&1 || exit $?
cd "$R" && python3 scripts/rocpd_step.py "$(ls gpurun_out/aa_prof/*/seg_results.db | head -n 1)" > gpurun_out/aa_segstep.md || exit 1
grep -E "s2d_rows|seghead|kernel total" gpurun_out/aa_segstep.md
rm -rf gpurun_out/aa_prof
