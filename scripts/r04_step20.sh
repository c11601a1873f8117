#!/bin/bash
# round 4: heavy batch width 6 vs 4 at the other shapes (R8 F = 8, the 20ng-shaped graph at F = 200 and 20)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
for v in product hu6 product hu6; do
  lib=""; [ $v != product ] && lib="GCNK_LIB=$PWD/_variants/libgcnk_$v.so"
  for g in r8:8 20ng:200,20; do
    env $lib timeout -k 10 200 python -u scripts/hub_probe.py --variants row --graph ${g%%:*} --widths ${g#*:} --reps 200 --mode cold > gpurun_out/r04/hu_$v.log 2>&1 || { echo "$v rc=$?"; exit 4; }
    grep "^{" gpurun_out/r04/hu_$v.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('$v', '${g%%:*}', d.get('width', d.get('F')), d['variant'], d['cold_us'], d['max_err'] < 1e-5)"
  done
done
