#!/bin/bash
# LDS counters of the hub group kernel (one --pmc pass, SQ block only).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES --output-format csv -d gpurun_out/r03/ldspmc -o pmc -- \
  python3 scripts/hub_probe.py --reps 20 --variants hub --widths 200 --mode cold > gpurun_out/r03/ldspmc.log 2>&1 || exit 3
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(list)
for f in glob.glob("gpurun_out/r03/ldspmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "hub_" in r["Kernel_Name"]:
            k = r["Kernel_Name"].split("::")[-1].split("(")[0]
            acc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{k:30s} {c:24s} mean {sum(v)/len(v):14.1f} n={len(v)}")
PY
