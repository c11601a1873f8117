#!/bin/bash
# Round 3, first GPU session of the hub plan: parity of the SpMM tests, then
# the north-star probe (row vs hub variants, warm / cold) and a rocprofv3
# kernel-trace summary of the cold hub rotation.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "spmm" > gpurun_out/r03/pytest_spmm.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/r03/pytest_spmm.log | tail -n 20
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/hub_probe.py --reps 200 > gpurun_out/r03/hub_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; cat gpurun_out/r03/hub_probe.log | grep -v amdgpu.ids
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03/kt_hub_cold -o kt -- \
  python -u scripts/hub_probe.py --reps 200 --variants hub --widths 200 --mode cold > gpurun_out/r03/kt_hub_cold.log 2>&1
rc=$?; echo "rocprof rc=$rc"
find gpurun_out/r03/kt_hub_cold -name "*kernel_stats.csv" -exec cat {} \;
exit $rc
