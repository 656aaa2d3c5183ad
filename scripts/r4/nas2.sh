#!/bin/bash
# Round-4 (session 2): NAS candidates/hour at 1 / 4 / 8 workers per GPU (32 CIFAR LeNet mutants x 5
# epochs, hipGraph steps) and the kernel census of a candidate run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/n2_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ]; then tail -20 "gpurun_out/n2_$name.log"; exit $rc; fi
  return $rc
}
for w in 1 4 8; do
  step nas_w$w 600 python3 bench/search_throughput.py --candidates 32 --epochs 5 --dataset cifar --graph on \
    --workers-per-device $w
  grep '^{' gpurun_out/n2_nas_w$w.log | cut -c1-300
done
rm -rf gpurun_out/sprof_n2
step nasprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sprof_n2 -o run -- \
  python3 bench/search_throughput.py --candidates 8 --epochs 1 --dataset cifar --graph on
python3 scripts/r4/nas_census.py gpurun_out/sprof_n2 > gpurun_out/n2_nas_census.md 2>&1; head -24 gpurun_out/n2_nas_census.md
