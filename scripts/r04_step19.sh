#!/bin/bash
# round 4: north-star heavy batch width (HEAVY_U) with one light row per wave
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
for v in ${VARIANTS:-product hu6 hu8 hu12}; do
  lib=""; [ $v != product ] && lib="GCNK_LIB=$PWD/_variants/libgcnk_$v.so"
  env $lib timeout -k 10 200 python -u scripts/hub_probe.py --variants row,light,topic --widths 200 --ipc ${IPC:-8,12,16} --reps 200 --mode cold > gpurun_out/r04/sweep3_$v.log 2>&1; echo "$v rc=$?"
  grep "^{" gpurun_out/r04/sweep3_$v.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('$v', d['variant'], d['ipc'], d['cold_us'], d['max_err'] < 1e-5, d['deterministic'])"
done
