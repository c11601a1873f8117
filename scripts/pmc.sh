#!/bin/bash
# HBM traffic per kernel of the R8 forward: two rocprofv3 --pmc passes (FETCH_SIZE
# uses 3 TCC counters, WRITE_SIZE 2: they cannot share a pass), each with its
# own time limit, then a per-kernel summary (scripts/pmc_summary.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/fetch -o run -- \
  python3 scripts/pmc_ops.py > gpurun_out/pmc/fetch.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/write -o run -- \
  python3 scripts/pmc_ops.py > gpurun_out/pmc/write.log 2>&1 || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.json && cat gpurun_out/pmc/summary.json
