#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for o in fp8 bf16; do
  rm -rf gpurun_out/p_$o
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_$o -o run -- \
    python3 bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 --steps 1 --warmup 0 --only $o > gpurun_out/p_$o.log 2>&1 || exit 1
  python3 scripts/prof_summary.py gpurun_out/p_$o/run_kernel_trace.csv --steps 1 > gpurun_out/r3_${o}_128_kernels.md 2>&1
  echo "== $o"; head -12 gpurun_out/r3_${o}_128_kernels.md
done
