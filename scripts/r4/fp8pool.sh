#!/bin/bash
# fp8 fused-pool row table (edge-coloured, conflict-free): numerics + 128^3 batch-1024 kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fp8_stem_gpu.py tests/test_kernels_gpu.py -k "f8 or fp8 or pool" -x -v -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/fp8pool_test.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/fp8pool_test.log
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/fprof2; mkdir -p gpurun_out/fprof2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fprof2 -o run -- \
  python3 bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 --steps 2 --warmup 1 > gpurun_out/fprof2.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep metric gpurun_out/fprof2.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
python3 - <<'PY' > gpurun_out/fprof2_kernels.md
import csv
rows = sorted(csv.DictReader(open("gpurun_out/fprof2/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
print("| us | kernel |\n|---|---|")
for r in rows[-12:]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"| {d:.1f} | `{r['Kernel_Name'][:70]}` |")
PY
cat gpurun_out/fprof2_kernels.md
