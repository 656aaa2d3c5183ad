#!/bin/bash
# Round-4 batch: tests of the new paths (seg fused loss, int8 stem), seg A/B, fp8 inference A/B
# (bf16 stem vs int8 stem), conv_tile32 PMC A/B, robustness path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_subpixel_gpu.py tests/test_fp8_stem_gpu.py > gpurun_out/b3_pytest.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/b3_pytest.log | head -20; tail -5 gpurun_out/b3_pytest.log; exit 1; }
tail -2 gpurun_out/b3_pytest.log
for st in 0 i8 0 i8; do
  FN_F8_STEM=$st timeout -k 10 300 python3 bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 > gpurun_out/b3_fp8_$st.log 2>&1 || { tail gpurun_out/b3_fp8_$st.log; exit 1; }
  echo "fp8 stem=$st"; grep '^{' gpurun_out/b3_fp8_$st.log | cut -c1-400
done
for x in 1 0 1 0; do
  FN_SEG_XENT=$x timeout -k 10 300 python3 bench.py --model seg --steps 10 --warmup 3 > gpurun_out/b3_seg.log 2>&1 || { tail gpurun_out/b3_seg.log; exit 1; }
  echo "seg xent=$x $(grep -o '"value": [0-9.]*' gpurun_out/b3_seg.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b3_seg.log)"
done
bash scripts/r4/m32_pmc.sh || exit $?
bash scripts/r4/robust.sh
