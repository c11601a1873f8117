#!/bin/bash
# One GPU-box session: parity tests, smoke, bench.  Stops at the first GPU
# fault / abort / timeout (exit codes other than 0 or 1 from pytest).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -v -p no:cacheprovider \
  --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -n 40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc2=$?; echo "smoke rc=$rc2"; tail -n 5 gpurun_out/smoke.log
if [ $rc2 -ne 0 ]; then exit $rc2; fi
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc3=$?; echo "bench rc=$rc3"; tail -n 5 gpurun_out/bench.log
exit $rc3
