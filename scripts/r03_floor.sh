#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
for m in cold warm; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03/floor_$m -o kt -- \
  python3 scripts/copy_floor.py --mode $m > gpurun_out/r03/floor_$m.log 2>&1 || exit 3
grep "^{" gpurun_out/r03/floor_$m.log
python3 - $m <<'PY'
import csv, glob, sys
for f in glob.glob(f"gpurun_out/r03/floor_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"  {r['Name'][:90]:90s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:7.2f} us  min {float(r['MinNs'])/1e3:7.2f}")
PY
done
