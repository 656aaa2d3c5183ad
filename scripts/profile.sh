#!/bin/bash
# rocprofv3 kernel-trace + stats of the native bench (per-kernel time).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
OUT=${OUT:-gpurun_out/prof}
timeout -k 10 ${PTIME:-600} rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 bench.py --steps ${STEPS:-5} --warmup 2 ${BENCH_ARGS:-} > gpurun_out/prof_bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_bench.log
find "$OUT" -name "*kernel_stats.csv" | head -3 | while read f; do echo "== $f"; head -40 "$f"; done
exit $rc
