#!/bin/bash
# round 4: heavy-row schedule sweep with nontemporal stores (topic rows alone + all rows, F = 200, cold)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
for v in product hu12w4 hu8w4 lwin; do
  lib=""; [ $v != product ] && lib="GCNK_LIB=$PWD/_variants/libgcnk_$v.so"
  env $lib timeout -k 10 200 python -u scripts/hub_probe.py --variants row,light,topic --widths 200 --ipc 12,16 --reps 200 --mode cold > gpurun_out/r04/sweep_$v.log 2>&1; echo "$v rc=$?"
  grep "^{" gpurun_out/r04/sweep_$v.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('$v', d['variant'], d['ipc'], d['cold_us'], d['max_err'] < 1e-5, d['deterministic'])"
done
