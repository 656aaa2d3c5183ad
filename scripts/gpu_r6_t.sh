#!/bin/bash
# Round 6: kernel traces of this tree and of the round-5 tree (abtest_old/) on one box, to find the
# kernels behind the same-box step difference.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/t_prof_new" -o step -- \
  python3 "$R/bench.py" --steps 5 --warmup 5 > "$R/gpurun_out/t_prof_new.log" 2>&1 || exit $?
echo new done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/t_prof_old" -o step -- \
  python3 "$R/abtest_old/bench.py" --steps 5 --warmup 5 > "$R/gpurun_out/t_prof_old.log" 2>&1 || exit $?
echo old done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/t_prof_new2" -o step -- \
  python3 "$R/bench.py" --steps 5 --warmup 5 > "$R/gpurun_out/t_prof_new2.log" 2>&1 || exit $?
echo new2 done
