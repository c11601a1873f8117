#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "spmm or graph_capture or gcn or trained" > gpurun_out/r03/pytest_hub.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 15 gpurun_out/r03/pytest_hub.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/variant_prof.sh "--variants row,hub --widths 200,8 --reps 200 --mode cold" base || exit 3
STAMP_WIDTHS=200 VARIANTS=stamps bash scripts/r03_stamps.sh
