#!/bin/bash
# GPU box: a subset of the GPU tests (-k expression in $1), stopping at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "$1" > gpurun_out/pytest_k.log 2>&1
rc=$?
tail -n 30 gpurun_out/pytest_k.log
exit $rc
