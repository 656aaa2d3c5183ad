#!/bin/bash
# Inference FC1 on 256-row dense workgroups: tests + 128^3 batch-1024 inference A/B (FN_DENSE_RT2 = old)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dense_infer_gpu.py tests/test_kernels_gpu.py -k "dense or linear or fp8" -x -q -m gpu \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fc1_test.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/fc1_test.log
[ $rc -eq 0 ] || exit $rc
for v in new old new; do
  if [ $v = old ]; then export FN_DENSE_RT2=1; else unset FN_DENSE_RT2; fi
  timeout -k 10 300 python3 bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 --steps 2 --warmup 1 > gpurun_out/fc1_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; grep metric gpurun_out/fc1_$v.log | grep -o '"precision": "[a-z0-9]*".*"ms_per_batch": [0-9.]*'
  [ $rc -eq 0 ] || exit $rc
done
unset FN_DENSE_RT2
rm -rf gpurun_out/fprof3; mkdir -p gpurun_out/fprof3
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fprof3 -o run -- \
  python3 bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 --steps 1 --warmup 1 --only fp8 > gpurun_out/fprof3.log 2>&1
echo "prof rc=$?"
python3 - <<'PY'
import csv
rows = sorted(csv.DictReader(open("gpurun_out/fprof3/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
for r in rows[-8:]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"{d:9.1f}  {r['Kernel_Name'][:70]}")
PY
