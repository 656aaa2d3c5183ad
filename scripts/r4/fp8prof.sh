#!/bin/bash
# fp8 128^3 inference (batch 1024, one chunk) kernel trace + fp8 parity (2 seeds)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
rm -rf gpurun_out/fprof; mkdir -p gpurun_out/fprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fprof -o run -- \
  python3 bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 --steps 1 --warmup 1 --only fp8 > gpurun_out/fprof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep metric gpurun_out/fprof.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
python3 - <<'PY' > gpurun_out/fprof_kernels.md
import csv
rows = sorted(csv.DictReader(open("gpurun_out/fprof/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
print("| us | kernel |\n|---|---|")
for r in rows[-16:]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"| {d:.1f} | `{r['Kernel_Name'][:70]}` |")
PY
cat gpurun_out/fprof_kernels.md
for seed in 0 1; do
  timeout -k 10 600 python3 bench/accuracy.py --epochs 16 --train-per-class 1000 --fp8 --seed $seed > gpurun_out/facc_$seed.log 2>&1
  echo "acc seed $seed rc=$?"; grep -o '"top1_bf16": [0-9.]*, "top1_fp8": [0-9.]*, "drop_pt": [-0-9.]*, "agreement": [0-9.]*' gpurun_out/facc_$seed.log | head -1
done
