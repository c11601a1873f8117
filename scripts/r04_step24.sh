#!/bin/bash
# round 4: B fragments prefetched from LDS ahead of the MFMAs (smallm, shortk, hubfactor phase 1)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -p no:cacheprovider -x -q --timeout 120 --timeout-method thread -k "small_m or factor or record or gemm or trained" > gpurun_out/r04/pytest_24.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r04/pytest_24.log
[ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/r04/pf_gemm.log
for shape in "50 200 7464:117" "70 200 100:0" "18846 200 100:0"; do
  GCNK_PROBE_SPLIT=${shape#*:} timeout -k 10 100 python -u scripts/gemm_probe.py ${shape%:*} >> gpurun_out/r04/pf_gemm.log 2>&1 || exit 4
done
grep "^{" gpurun_out/r04/pf_gemm.log
timeout -k 10 200 python -u scripts/factor_probe.py > gpurun_out/r04/pf_factor.log 2>&1; echo "probe rc=$?"; grep "^{" gpurun_out/r04/pf_factor.log
GCNK_FACTOR_XHUB=gemm timeout -k 10 200 python -u scripts/factor_probe.py --graphs r8 > gpurun_out/r04/pf_factor_gemm.log 2>&1; echo "probe rc=$?"; grep "^{" gpurun_out/r04/pf_factor_gemm.log
