#!/bin/bash
# GPU box: north-star microbenchmark (scripts/micro/ns_micro.hip, built in-tree beforehand).
# usage: run_ns_micro.sh [SEG] ; NS_ONLY=<substring> selects variants; PROF=1 adds a rocprofv3 kernel-stats pass
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/micro
python3 scripts/micro/dump_r8.py /tmp/r8_adj.bin || exit 3
timeout -k 10 120 scripts/micro/ns_micro /tmp/r8_adj.bin "${1:-128}" > gpurun_out/micro/ns.log 2>&1 || { echo "rc=$?"; cat gpurun_out/micro/ns.log; exit 3; }
cat gpurun_out/micro/ns.log
if [ -n "$PROF" ]; then
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/micro/nsprof -o kt -- scripts/micro/ns_micro /tmp/r8_adj.bin "${1:-128}" > gpurun_out/micro/nsprof.log 2>&1 || { echo "prof rc=$?"; tail gpurun_out/micro/nsprof.log; exit 3; }
  python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/micro/nsprof/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"  {r['Name'][:90]:90s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:7.2f} us  min {float(r['MinNs'])/1e3:7.2f}")
PY
fi
