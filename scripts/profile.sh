#!/bin/bash
# rocprofv3 kernel-trace summary of the bench command (no PMC here).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 bench.py --steps ${STEPS:-100} --warmup 10 --cpu-sample-s 0 ${BENCH_ARGS} > gpurun_out/prof/bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"; tail -n 3 gpurun_out/prof/bench.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
