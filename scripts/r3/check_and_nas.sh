#!/bin/bash
# GPU suite + smoke + bench, then the NAS census workload (scripts/r3/nas.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
SKIP_TORCH=1 STEPS=20 bash scripts/gpu_check.sh || exit $?
bash scripts/r3/nas.sh
