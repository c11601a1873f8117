#!/bin/bash
# GPU box: run one prebuilt standalone microbenchmark of scripts/micro on the R8 A-hat.
# usage: run_micro.sh <binary> [args...] ; NS_ONLY=<substring> selects variants;
#        PROF=1 adds a rocprofv3 kernel-stats pass.  Output: gpurun_out/micro/<binary>.log
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
bin="$1"; shift
mkdir -p gpurun_out/micro
python3 scripts/micro/dump_r8.py /tmp/r8_adj.bin || exit 3
timeout -k 10 240 "scripts/micro/$bin" /tmp/r8_adj.bin "$@" > "gpurun_out/micro/$bin.log" 2>&1 || { echo "rc=$?"; cat "gpurun_out/micro/$bin.log"; exit 3; }
cat "gpurun_out/micro/$bin.log"
if [ -n "$PROF" ]; then
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/micro/${bin}_prof" -o kt -- "scripts/micro/$bin" /tmp/r8_adj.bin "$@" > "gpurun_out/micro/${bin}_prof.log" 2>&1 || { echo "prof rc=$?"; tail "gpurun_out/micro/${bin}_prof.log"; exit 3; }
  python3 - "$bin" <<'PY'
import csv, glob, sys
for f in glob.glob(f"gpurun_out/micro/{sys.argv[1]}_prof/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"  {r['Name'][:90]:90s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:7.2f} us  min {float(r['MinNs'])/1e3:7.2f}")
PY
fi
