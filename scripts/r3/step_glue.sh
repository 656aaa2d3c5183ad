#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
timeout -k 10 300 python3 scripts/r3/step_glue_probe.py 2>&1 | grep -v amdgpu.ids | tail -40
