#!/bin/bash
# hub_stamps.py timeline under each prebuilt stamps variant (_variants/libgcnk_<name>.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
ARGS="$1"; shift
mkdir -p gpurun_out
for V in "$@"; do
  echo "== $V"
  GCNK_LIB=$PWD/_variants/libgcnk_$V.so timeout -k 10 120 python -u scripts/hub_stamps.py $ARGS > gpurun_out/stamps_$V.log 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/stamps_$V.log; exit 3; }
  grep '^{' gpurun_out/stamps_$V.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print('  F=%d entry p50 %.2f p100 %.2f | record %.2f | stage %.2f | outputs p0 %.2f p50 %.2f p100 %.2f | light_end p50 %.2f p100 %.2f | finish entry %.2f sum %.2f end %.2f' % (
      d['F'], d['light_entry']['p50'], d['light_entry']['p100'], d['record']['p50'], d['stage']['p50'], d['outputs']['p0'], d['outputs']['p50'], d['outputs']['p100'],
      d['light_end']['p50'], d['light_end']['p100'], d['finish_entry']['p50'], d['finish_sum']['p50'], d['finish_end']['p100']))"
done
