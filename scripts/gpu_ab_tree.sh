#!/bin/bash
# A/B of the training (and seg) step: this tree vs a prebuilt older tree in abtest_old/, alternating
# on one box (3 runs each for the classifier, 2 for seg)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/abt_new$i.log 2>&1 || exit $?
  echo "new$i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abt_new$i.log)"
  (cd abtest_old && timeout -k 10 200 python bench.py --steps 30 --warmup 5 > ../gpurun_out/abt_old$i.log 2>&1) || exit $?
  echo "old$i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abt_old$i.log)"
done
for i in 1 2; do
  timeout -k 10 200 python bench.py --model seg --steps 10 --warmup 3 > gpurun_out/abt_snew$i.log 2>&1 || exit $?
  echo "seg new$i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abt_snew$i.log)"
  (cd abtest_old && timeout -k 10 200 python bench.py --model seg --steps 10 --warmup 3 > ../gpurun_out/abt_sold$i.log 2>&1) || exit $?
  echo "seg old$i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abt_sold$i.log)"
done
