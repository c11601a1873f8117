#!/bin/bash
# L1 (TCP) / L2 (TCC) counter passes over a probe command, one rocprofv3 --pmc
# run each under its own time limit; per-kernel means -> gpurun_out/cache/summary.txt
# usage: bash scripts/cache_pmc.sh "<python args after python3>"
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
CMD="$1"
mkdir -p gpurun_out/cache
i=0
for P in "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum" \
         "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum" \
         "TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_READ_sum TCC_WRITE_sum" \
         "TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum TD_BUSY_avr"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/cache/p$i -o run -- python3 $CMD > gpurun_out/cache/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -3 gpurun_out/cache/p$i.log; }
done
python3 - <<'PY' | tee gpurun_out/cache/summary.txt
import csv, glob
from collections import defaultdict
vals = defaultdict(list)
for f in glob.glob("gpurun_out/cache/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "spmm_row_kernel" not in n and "hub_" not in n and "tile" not in n:
            continue
        n = n.split("(anonymous namespace)::")[-1].split("(")[0]
        vals[(n, r["Counter_Name"])].append(float(r["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    print(f"{k[0]:60s} {k[1]:34s} {sum(v)/len(v):14.1f}  (n={len(v)})")
PY
