#!/bin/bash
# For each prebuilt _variants/libgcnk_<name>.so (or "base" = the in-tree library):
# time the north-star op with scripts/hub_probe.py and take the rocprofv3
# kernel-trace average of every gcnk kernel it launched.
# usage: bash scripts/variant_prof.sh "<probe args>" name1 name2 ...
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
ARGS="$1"; shift
mkdir -p gpurun_out/vprof
for V in "$@"; do
  if [ "$V" = base ]; then unset GCNK_LIB; else export GCNK_LIB=$PWD/_variants/libgcnk_$V.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vprof/$V -o run -- \
    python3 ${PROBE:-scripts/hub_probe.py} $ARGS > gpurun_out/vprof/$V.log 2>&1 || { echo "$V failed rc=$?"; tail -5 gpurun_out/vprof/$V.log; exit 3; }
  echo "== $V"
  grep "^{" gpurun_out/vprof/$V.log | grep -v variant; grep "\"variant\"" gpurun_out/vprof/$V.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('  F=%d %s warm %.2f us cold %.2f us err %.1e blocks %d' % (d['F'], d['variant'], d['warm_us'], d['cold_us'], d['max_err'], d['hdr'][4]))"
  python3 - "$V" <<'PY'
import csv, glob, sys
for f in glob.glob(f"gpurun_out/vprof/{sys.argv[1]}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gcnk" in r["Name"]:
            n = r["Name"].split("(anonymous namespace)::")[-1].split("(")[0]
            print(f"  {n:45s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:7.2f} us  min {float(r['MinNs'])/1e3:7.2f}")
PY
done
