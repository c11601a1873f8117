#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "bwd2 or gcn or train or trained or graph_convolution or dropout" > gpurun_out/r03/pytest_bwd.log 2>&1 || { echo "pytest rc=$?"; grep -E "Error|error|FAILED|assert" gpurun_out/r03/pytest_bwd.log | head -20; tail -3 gpurun_out/r03/pytest_bwd.log; exit 3; }
tail -2 gpurun_out/r03/pytest_bwd.log
bash scripts/r03_train.sh
