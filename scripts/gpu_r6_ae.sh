#!/bin/bash
# Round 6: kernel traces of the classifier step with FN_TILE_NT4=1 / 0 on one box (which
# 64-column convs gain from 64-column workgroups).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for f in 1 0; do
  cd /tmp && FN_TILE_NT4=$f timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/ae_prof_$f" -o step -- \
    python3 "$R/bench.py" --steps 5 --warmup 5 > "$R/gpurun_out/ae_prof_$f.log" 2>&1 || exit $?
  echo "prof $f done"
done
