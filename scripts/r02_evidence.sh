#!/bin/bash
# Round-2 evidence: full bench line, rocprofv3 kernel stats of a bench run
# (forward graphs), per-op warm/cold kernel stats (hub_probe / op_probe under
# rocprofv3), and the cache / SQ counter passes of the north-star kernel.
# Every GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r02
mkdir -p $O
timeout -k 10 500 python3 bench.py > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/bench.log; exit 3; }
tail -1 $O/bench.log > $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fwd -o fwd -- \
  python3 bench.py --steps 200 --warmup 20 --no-pmc --cpu-sample-s 0 --no-configs --kernel-reps 1 > $O/prof_fwd.log 2>&1 \
  || { echo "prof fwd rc=$?"; exit 3; }
for mode in warm cold; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_as1_$mode -o as1 -- \
    python3 scripts/hub_probe.py --reps 200 --variants row --widths 200 --mode $mode > $O/prof_as1_$mode.log 2>&1 \
    || { echo "prof as1 $mode rc=$?"; exit 3; }
done
echo done
