#!/bin/bash
# GPU box: R8 push-schedule microbenchmark (scripts/micro/hub_micro.hip, built in-tree beforehand).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/micro
python3 scripts/micro/dump_r8.py /tmp/r8_adj.bin || exit 3
for cfg in "${@:-32,7}"; do
  set -- ${cfg/,/ }
  timeout -k 10 60 scripts/micro/hub_micro /tmp/r8_adj.bin $1 $2 > gpurun_out/micro/hub_$1_$2.log 2>&1 || { echo "rc=$? cfg $cfg"; cat gpurun_out/micro/hub_$1_$2.log; exit 3; }
  cat gpurun_out/micro/hub_$1_$2.log
done
if [ -n "$PROF" ]; then
  set -- ${PROF/,/ }
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/micro/prof -o kt -- scripts/micro/hub_micro /tmp/r8_adj.bin $1 $2 > gpurun_out/micro/prof.log 2>&1 || { echo "prof rc=$?"; tail gpurun_out/micro/prof.log; exit 3; }
  python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/micro/prof/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"  {r['Name'][:70]:70s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:7.2f} us  min {float(r['MinNs'])/1e3:7.2f}")
PY
fi
