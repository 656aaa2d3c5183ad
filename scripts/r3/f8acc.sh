#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 bench/accuracy.py --fp8 --epochs ${EP:-16} --train-per-class 1000 > gpurun_out/r3_acc_fp8.log 2>&1
rc=$?; tail -1 gpurun_out/r3_acc_fp8.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['val_acc_per_epoch'], d['fp8'])"; exit $rc
