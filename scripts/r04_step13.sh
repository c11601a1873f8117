#!/bin/bash
# round 4: persistent hubfactor with W1 staged once through LDS and the next block prefetched (20ng)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -p no:cacheprovider -x -q --timeout 120 --timeout-method thread -k "factor or 20ng or record" > gpurun_out/r04/pytest_13.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/r04/pytest_13.log
timeout -k 10 200 python -u scripts/factor_probe.py > gpurun_out/r04/fp20_v2.log 2>&1; echo "probe rc=$?"
grep "^{" gpurun_out/r04/fp20_v2.log
GCNK_STAMP_GRAPH=20ng GCNK_LIB=$PWD/_variants/libgcnk_stamps.so timeout -k 10 120 python -u scripts/factor_stamps.py > gpurun_out/r04/factorstamps20v2.log 2>&1; echo "stamps rc=$?"
grep "^{" gpurun_out/r04/factorstamps20v2.log | cut -c1-900
