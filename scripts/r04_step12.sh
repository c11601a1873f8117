#!/bin/bash
# round 4: full GPU suite + smoke + the default bench line, saving the rocprof summaries
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04/bench_prof
timeout -k 10 600 python -u -m pytest tests/ -m gpu -p no:cacheprovider -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_final.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r04/pytest_final.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04/smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/r04/smoke.log
timeout -k 10 600 python -u bench.py --rocprof-dir gpurun_out/r04/bench_prof > gpurun_out/r04/bench_final.log 2>&1; echo "bench rc=$?"
tail -c 1500 gpurun_out/r04/bench_final.log
