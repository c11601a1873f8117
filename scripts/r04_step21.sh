#!/bin/bash
# round 4: X_hubs W1 at R8's shape (50 dense hub rows x 7463, F = 200): tile SpMM vs split-K GEMM
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
GCNK_FACTOR_XHUB=gemm timeout -k 10 200 python -u scripts/factor_probe.py --graphs r8 > gpurun_out/r04/xhub_gemm.log 2>&1; echo "probe rc=$?"; grep "^{" gpurun_out/r04/xhub_gemm.log
for s in 16 32 64 128; do
  GCNK_PROBE_SPLIT=$s timeout -k 10 100 python -u scripts/gemm_probe.py 50 200 7463 >> gpurun_out/r04/xhub_gemm.log 2>&1 || exit 4
done
grep "^{" gpurun_out/r04/xhub_gemm.log | tail -4
