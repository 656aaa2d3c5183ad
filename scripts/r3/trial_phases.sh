#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
timeout -k 10 400 python3 scripts/r3/trial_phases.py 2>&1 | grep -v amdgpu.ids | tail -15
