#!/bin/bash
# 128^3 inference (bf16 and fp8) under rocprofv3 --kernel-trace --stats; TPC>0 also runs the
# trained-model fp8 parity of bench/accuracy.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/iprof; mkdir -p gpurun_out/iprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/iprof -o run -- \
  python3 bench/infer_fp8.py --size 128 --batch 256 --chunk 128 --steps 1 --warmup 1 > gpurun_out/iprof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep metric gpurun_out/iprof.log
[ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import csv
rows = sorted(csv.DictReader(open("gpurun_out/iprof/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
for r in rows[-14:]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(round(d, 1), r["Kernel_Name"][:60])
PY
if [ "${TPC:-0}" -gt 0 ]; then
  timeout -k 10 400 python3 bench/accuracy.py --train-per-class $TPC --epochs 10 --fp8 > gpurun_out/acc_fp8.log 2>&1
  rc=$?; tail -1 gpurun_out/acc_fp8.log
fi
exit $rc
