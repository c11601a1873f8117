#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
for V in ${VARIANTS:-stamps}; do
  GCNK_LIB=$PWD/_variants/libgcnk_$V.so timeout -k 10 120 python -u scripts/hub_stamps.py ${STAMP_ARGS:-0} > gpurun_out/r03/stamps_$V.log 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/r03/stamps_$V.log; exit 3; }
  echo "== stamps $V"; grep "^{" gpurun_out/r03/stamps_$V.log
done
