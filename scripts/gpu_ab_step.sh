#!/bin/bash
# A/B of the training step: this tree vs a prebuilt older tree in abtest_old/ (bench twice each,
# alternating), then a rocprofv3 kernel trace of this tree's bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/ab_new$i.log 2>&1 || exit $?
  echo "new$i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_new$i.log)"
  (cd abtest_old && timeout -k 10 200 python bench.py --steps 30 --warmup 5 > ../gpurun_out/ab_old$i.log 2>&1) || exit $?
  echo "old$i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_old$i.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab_prof -o run -- \
  python3 bench.py --steps 5 --warmup 2 > gpurun_out/ab_prof.log 2>&1 || exit $?
timeout -k 10 120 python scripts/diag_step_kernels.py --small-us 20 > gpurun_out/ab_diag.log 2>&1; tail -2 gpurun_out/ab_diag.log
timeout -k 10 120 python scripts/diag_nas_step.py --list > gpurun_out/ab_nas.log 2>&1; tail -1 gpurun_out/ab_nas.log
FN_F8_BLOCK=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ab_f8 -o run -- \
  python3 bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 --only fp8 --steps 1 --warmup 1 > gpurun_out/ab_f8.log 2>&1 || exit $?
exit 0
