#!/bin/bash
# Segmentation head bench + step trace; same-box stock-PyTorch and native headline runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --model seg --steps 10 --warmup 3 > gpurun_out/seg_bench.log 2>&1 || { tail -20 gpurun_out/seg_bench.log; exit 1; }
grep '^{' gpurun_out/seg_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('seg', d['value'], d['ms_per_step'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/seg_prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --model seg --steps 3 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/seg_prof.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT"
if [ "${TORCH:-1}" = "1" ]; then
timeout -k 10 600 python bench.py --impl torch --torch-find --steps 20 --warmup 5 > gpurun_out/r3_torch.log 2>&1 || { tail -20 gpurun_out/r3_torch.log; exit 1; }
grep '^{' gpurun_out/r3_torch.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('torch', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_native_same_box.log 2>&1 || { tail -20 gpurun_out/r3_native_same_box.log; exit 1; }
grep '^{' gpurun_out/r3_native_same_box.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('native', d['value'], d['ms_per_step'])"
fi
