#!/bin/bash
# conv_wtile diagnostics: loader ablations (FN_WTILE_DBG 4 = no x-halo DMA, 8 = no dy DMA;
# timing only) and one PMC pass (L2 hits / misses, HBM fetch) over the layer bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in ${DBGS:-4 8 12}; do
  FN_WTILE_DBG=$d timeout -k 10 200 python -u scripts/bench_conv_layers.py --batch 128 --reps 10 --only conv2,conv3,conv4 \
    > gpurun_out/wtd$d.log 2>&1 || exit 1
  echo "== dbg $d"; grep -oE "\"layer\": \"[a-z0-9_]+\"|\"wtile_wgrad_us\": [0-9.]+" gpurun_out/wtd$d.log
done
rm -rf gpurun_out/wpmc
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --kernel-trace --output-format csv -d gpurun_out/wpmc -o pmc -- \
  python3 scripts/bench_conv_layers.py --batch 128 --reps 2 --only conv2,conv3,conv4 > gpurun_out/wpmc.log 2>&1
echo "pmc rc=$?"
python3 - <<'PY'
import csv, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open([__import__('glob').glob('gpurun_out/wpmc/**/*counter_collection.csv', recursive=True)][0][0])):
    n = r["Kernel_Name"]
    if "wgrad" in n or "wtile" in n:
        agg[n[:40] + " " + r["Grid_Size"]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in agg.items():
    h, m = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
    print(k, "L2 hit %.3f" % (h / max(h + m, 1)), "L2 misses %.0f" % m, "TCP->TCC reads %.0f" % c.get("TCP_TCC_READ_REQ_sum", 0))
PY
