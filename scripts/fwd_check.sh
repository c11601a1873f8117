#!/bin/bash
# GPU box: targeted GPU tests ($1 = -k expression), then the forward's kernel timeline
# (rocprofv3 kernel trace of scripts/fwd_trace.py: a hipGraph of 10 R8 eval forwards).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/fwd
if [ -n "$1" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread -k "$1" > gpurun_out/pytest_k.log 2>&1 || { tail -n 40 gpurun_out/pytest_k.log; exit 3; }
  tail -n 2 gpurun_out/pytest_k.log
fi
rm -rf gpurun_out/fwd/trace
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fwd/trace -o fwd -- \
  python3 scripts/fwd_trace.py > gpurun_out/fwd/run.log 2>&1 || { echo "trace rc=$?"; tail gpurun_out/fwd/run.log; exit 4; }
python3 scripts/fwd_trace.py --report gpurun_out/fwd/trace
