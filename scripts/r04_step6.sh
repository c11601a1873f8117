#!/bin/bash
# round 4: in-kernel timelines (stamps build): the row plan at F = 200 / 8, the factored gc1
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
GCNK_LIB=$PWD/_variants/libgcnk_stamps.so timeout -k 10 120 python -u scripts/row_stamps.py 200 8 > gpurun_out/r04/rowstamps.log 2>&1; echo "rowstamps rc=$?"
grep "^{" gpurun_out/r04/rowstamps.log | cut -c1-1500
GCNK_LIB=$PWD/_variants/libgcnk_stamps.so timeout -k 10 120 python -u scripts/factor_stamps.py > gpurun_out/r04/factorstamps.log 2>&1; echo "factorstamps rc=$?"
tail -5 gpurun_out/r04/factorstamps.log | cut -c1-1500
