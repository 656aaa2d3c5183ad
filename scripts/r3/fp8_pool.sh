#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_fp8_stem_gpu.py tests/test_kernels_gpu.py -k "fp8" > gpurun_out/fp8p_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/fp8p_tests.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/fp8p_tests.log | head -20; exit $rc; }
FN_F8_POOL=0 timeout -k 10 300 python3 bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 --steps 3 --warmup 1 --only fp8 > gpurun_out/fp8p_nopool.log 2>&1 || { tail gpurun_out/fp8p_nopool.log; exit 1; }
grep '^{' gpurun_out/fp8p_nopool.log
PROF=1 ACC=0 bash scripts/r3/fp8.sh
python3 - <<'PY'
import csv
tr=list(csv.DictReader(open('gpurun_out/fp8prof/run_kernel_trace.csv')))
tr.sort(key=lambda r:int(r['Start_Timestamp']))
for r in tr[-12:]:
    d=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6
    print(f"{d:7.2f} ms {r['Grid_Size_X']:>9}x{r['Grid_Size_Y']} {r['Kernel_Name'][:70]}")
PY
