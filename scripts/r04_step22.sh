#!/bin/bash
# round 4: small-M split-K GEMM for X[hubs] W1 -- parity, then per-call time by k chunk and in the forward
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -p no:cacheprovider -x -q --timeout 120 --timeout-method thread -k "small_m or factor or record or gemm" > gpurun_out/r04/pytest_22.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r04/pytest_22.log
[ $rc -eq 0 ] || exit $rc
for s in 59 117 234 467; do
  GCNK_PROBE_SPLIT=$s timeout -k 10 100 python -u scripts/gemm_probe.py 50 200 7464 >> gpurun_out/r04/smallm.log 2>&1 || exit 4
done
grep "^{" gpurun_out/r04/smallm.log
timeout -k 10 200 python -u scripts/factor_probe.py > gpurun_out/r04/factor_probe22.log 2>&1; echo "probe rc=$?"; grep "^{" gpurun_out/r04/factor_probe22.log
