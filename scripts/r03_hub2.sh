#!/bin/bash
# Hub plan: workgroup size variants (rocprof kernel averages, cold rotation) and
# in-kernel stamps.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
bash scripts/variant_prof.sh "--variants hub --widths 200,8 --reps 200 --mode cold" base b512 b256 || exit $?
for V in stamps; do
  GCNK_LIB=$PWD/_variants/libgcnk_$V.so timeout -k 10 120 python -u scripts/hub_stamps.py 0 > gpurun_out/r03/stamps_$V.log 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/r03/stamps_$V.log; exit 3; }
  echo "== stamps $V"; grep "^{" gpurun_out/r03/stamps_$V.log
done
