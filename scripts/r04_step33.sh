#!/bin/bash
# round 4: default segment sizes re-checked after RPW = 1 / HEAVY_U = 6 (20ng-shaped F = 200, R8 F = 8)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
for rep in 1 2; do
  timeout -k 10 200 python -u scripts/hub_probe.py --variants row --graph 20ng --widths 200 --ipc 12,16,20,24,32 --reps 200 --mode cold > gpurun_out/r04/ipc20_$rep.log 2>&1 || exit 4
  timeout -k 10 200 python -u scripts/hub_probe.py --variants row --graph r8 --widths 8 --ipc 4,8,12,16 --reps 200 --mode cold > gpurun_out/r04/ipc8_$rep.log 2>&1 || exit 4
  cat gpurun_out/r04/ipc20_$rep.log gpurun_out/r04/ipc8_$rep.log | grep "^{" | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print($rep, d['graph'], d['F'], d['ipc'], d['cold_us'], d['max_err'] < 1e-5)"
done
