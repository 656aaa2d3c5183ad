#!/bin/bash
# Round-end check on the final tree, the way the driver runs it: the whole GPU suite (-x), the
# smoke step, the 1-GPU bench twice, the seg bench, and a kernel trace of the training step
# (rocprofv3 --kernel-trace --stats) for profiles/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/f_pytest.log 2>&1; rc=$?
tail -1 gpurun_out/f_pytest.log; grep -E "^FAILED|^ERROR" gpurun_out/f_pytest.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f_smoke.log 2>&1 || { tail -5 gpurun_out/f_smoke.log; exit 1; }
echo "smoke ok: $(tail -1 gpurun_out/f_smoke.log | cut -c1-200)"
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/f_bench$i.log 2>&1 || exit $?
  tail -1 gpurun_out/f_bench$i.log | cut -c1-250
done
timeout -k 10 300 python bench.py --model seg --steps 10 --warmup 3 > gpurun_out/f_seg.log 2>&1 || exit $?
tail -1 gpurun_out/f_seg.log | cut -c1-250
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/f_prof" -o step -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/f_prof.log" 2>&1
echo "prof rc=$?"
