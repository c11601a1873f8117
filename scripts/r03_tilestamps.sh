#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
GCNK_LIB=$PWD/_variants/libgcnk_stamps.so timeout -k 10 120 python -u scripts/tile_stamps.py > gpurun_out/r03/tilestamps.log 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/r03/tilestamps.log; exit 3; }
grep "^{" gpurun_out/r03/tilestamps.log
