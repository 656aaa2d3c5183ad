#!/bin/bash
# Round 6: kernel traces of this tree and the prebuilt older tree in abtest_old/ on one box
# (classifier and seg steps): which kernels the bf16 pair packing and the seghead lean instance moved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for t in new old; do
  B=$R; [ $t = old ] && B=$R/abtest_old
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/x_prof_$t" -o step -- \
    python3 "$B/bench.py" --steps 5 --warmup 5 > "$R/gpurun_out/x_prof_$t.log" 2>&1 || exit $?
  echo "prof $t done"
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/x_seg_$t" -o seg -- \
    python3 "$B/bench.py" --model seg --steps 5 --warmup 5 > "$R/gpurun_out/x_seg_$t.log" 2>&1 || exit $?
  echo "seg $t done"
done
cd "$R"
for t in new old; do
  python3 scripts/rocpd_step.py "$(ls gpurun_out/x_prof_$t/*/step_results.db gpurun_out/x_prof_$t/step_results.db 2>/dev/null | head -n 1)" > gpurun_out/x_step_$t.md || exit 1
  python3 scripts/rocpd_step.py "$(ls gpurun_out/x_seg_$t/*/seg_results.db gpurun_out/x_seg_$t/seg_results.db 2>/dev/null | head -n 1)" > gpurun_out/x_segstep_$t.md || exit 1
  tail -n 1 gpurun_out/x_step_$t.md; tail -n 1 gpurun_out/x_segstep_$t.md
done
rm -rf gpurun_out/x_prof_new gpurun_out/x_prof_old gpurun_out/x_seg_new gpurun_out/x_seg_old
