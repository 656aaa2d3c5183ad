#!/bin/bash
# NAS search throughput (MNIST + CIFAR LeNet-5 mutants) and a rocprofv3 kernel census of a
# CIFAR candidate run: which kernels are native, which come from torch / hipBLASLt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 bench/search_throughput.py --candidates 8 > gpurun_out/search_mnist.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/search_throughput.py --candidates 8 --dataset cifar > gpurun_out/search_cifar.log 2>&1 || exit $?
grep metric gpurun_out/search_mnist.log gpurun_out/search_cifar.log
rm -rf gpurun_out/sprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sprof -o run -- \
  python3 bench/search_throughput.py --candidates 4 --dataset cifar > gpurun_out/sprof.log 2>&1
echo "rocprof rc=$?"
python3 - <<'PY'
import csv, glob, collections, sys
sys.path.insert(0, "scripts")
from prof_summary import short
f = glob.glob("gpurun_out/sprof/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
cat = collections.defaultdict(float)
out = []
for r in rows:
    n = short(r["Name"]); t = float(r["TotalDurationNs"]) / 1e6
    k = "hipblaslt" if n.startswith("hipblaslt") else ("torch" if n.startswith("torch") or "at::" in r["Name"] else "native")
    cat[k] += t
    out.append((t, k, n, r["Calls"]))
tot = sum(cat.values())
print("kernel time by origin (ms):", {k: round(v, 2) for k, v in cat.items()}, "total", round(tot, 2))
for t, k, n, c in sorted(out, reverse=True)[:25]:
    print(f"{t:9.3f} ms  {k:9s} {c:>6s}  {n}")
PY
