#!/bin/bash
# round 4: gcn_bwd2 in-kernel timeline at R8's shape
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
GCNK_LIB=$PWD/_variants/libgcnk_stamps.so timeout -k 10 120 python -u scripts/bwd2_stamps.py > gpurun_out/r04/bwd2_stamps.log 2>&1; echo "stamps rc=$?"
grep "^{" gpurun_out/r04/bwd2_stamps.log
