#!/bin/bash
# round 4: persistent hubfactor coarse timeline (20ng): entry, first block staged, first block done, exit
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
GCNK_STAMP_GRAPH=20ng GCNK_LIB=$PWD/_variants/libgcnk_stamps.so timeout -k 10 120 python -u scripts/factor_stamps.py > gpurun_out/r04/factorstamps20c.log 2>&1; echo "factorstamps20 rc=$?"
grep "^{" gpurun_out/r04/factorstamps20c.log | cut -c1-1500
timeout -k 5 60 scripts/micro/xcc_map > gpurun_out/r04/xcc_map.log 2>&1; echo "xcc rc=$?"
cat gpurun_out/r04/xcc_map.log
