#!/bin/bash
# After a kernel change on the training step: the tests it touches (TESTS), two benches and a
# kernel trace of the step (rocpd_step.py summarises it)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS=${TESTS:-"tests/test_kernels_gpu.py tests/test_determinism_gpu.py tests/test_conv_wtile_gpu.py"}
timeout -k 10 900 python -u -m pytest $TESTS -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/cs_tests.log 2>&1; rc=$?
tail -1 gpurun_out/cs_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/cs_tests.log | head
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/cs_bench$i.log 2>&1 || exit $?
  tail -1 gpurun_out/cs_bench$i.log | cut -c1-160
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/cs_prof" -o step -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/cs_prof.log" 2>&1
echo "prof rc=$?"
cd "$GRAFT_REPO_ROOT" && [ -n "${NAS:-}" ] && bash scripts/gpu_nas_scale.sh
exit 0
