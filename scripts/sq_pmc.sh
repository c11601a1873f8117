#!/bin/bash
# SQ / SQC counter passes (one rocprofv3 --pmc run each, its own time limit) over
# a probe command; per-kernel means -> gpurun_out/sq/summary.txt
# usage: bash scripts/sq_pmc.sh "<python args after python3>"
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
CMD="$1"
mkdir -p gpurun_out/sq
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_LDS" \
         "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQC_ICACHE_MISSES_DUPLICATE" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS" \
         "SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/sq/p$i -o run -- python3 $CMD > gpurun_out/sq/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -3 gpurun_out/sq/p$i.log; exit 3; }
done
python3 - <<'PY' | tee gpurun_out/sq/summary.txt
import csv, glob
from collections import defaultdict
vals = defaultdict(list)
for f in glob.glob("gpurun_out/sq/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "gcnk" not in n:
            continue
        n = n.split("(anonymous namespace)::")[-1].split("(")[0]
        vals[(n, r["Counter_Name"])].append(float(r["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    print(f"{k[0]:40s} {k[1]:30s} {sum(v)/len(v):14.1f}  (n={len(v)})")
PY
