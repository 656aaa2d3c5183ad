#!/bin/bash
# Round-4 batch: seg fused head+loss (tests + bench A/B), conv_tile32 PMC A/B, robustness path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_subpixel_gpu.py > gpurun_out/b2_pytest.log 2>&1 || { tail -30 gpurun_out/b2_pytest.log; exit 1; }
tail -3 gpurun_out/b2_pytest.log
for x in 1 0 1 0; do
  FN_SEG_XENT=$x timeout -k 10 300 python3 bench.py --model seg --steps 10 --warmup 3 > gpurun_out/b2_seg.log 2>&1 || { tail gpurun_out/b2_seg.log; exit 1; }
  echo "seg xent=$x $(grep -o '"value": [0-9.]*' gpurun_out/b2_seg.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b2_seg.log)"
done
bash scripts/r4/m32_pmc.sh || exit $?
bash scripts/r4/robust.sh
