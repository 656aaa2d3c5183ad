#!/bin/bash
# End-to-end NAS on one MI355X through the CLI: FullEvolution from the lenet5 template, CIFAR-shaped
# synthetic data, 32 individuals, 5 training epochs, 3 evolution generations, CW + PGD robustness
# on every candidate, auto workers (4 per GPU, a pool that persists across generations); the
# history line carries each generation's trial wall time
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf /tmp/fn_nas_run
timeout -k 10 900 python -m featurenet_amd.cli run -n 32 -t 5 -e 3 -d cifar -l lenet5 --seed 0 -b /tmp/fn_nas_run \
  > gpurun_out/evo.log 2>&1; rc=$?
grep -v "^/opt" gpurun_out/evo.log | tail -4 | cut -c1-1500
exit $rc
