#!/bin/bash
# The data-parallel step on one GPU: bucketed RCCL all-reduce (world-1 communicator) captured
# in the step graph, against the plain step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for a in "" "--force-allreduce"; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 5 $a > gpurun_out/far.log 2>&1 || { tail -20 gpurun_out/far.log; exit 1; }
  grep '^{' gpurun_out/far.log | python3 -c "import json,sys; [print('args [$a]', (d:=json.loads(l))['value'], d['ms_per_step'], 'graph', d['config']['graph'], 'fallback', d['graph_fallback'], 'loss', d['final_loss'], d['dist']) for l in sys.stdin]"
done
