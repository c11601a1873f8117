#!/bin/bash
# round 4: short-K / small-M GEMMs with and without the LDS fragment prefetch (old = previous commit)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
rm -f gpurun_out/r04/pf2.log
for v in old product old product; do
  lib=""; [ $v != product ] && lib="GCNK_LIB=$PWD/_variants/libgcnk_$v.so"
  for shape in "50 200 7464:117" "70 200 100:0" "18846 200 100:0" "300 200 100:0"; do
    env $lib GCNK_PROBE_SPLIT=${shape#*:} timeout -k 10 100 python -u scripts/gemm_probe.py ${shape%:*} > gpurun_out/r04/pf2_one.log 2>&1 || exit 4
    echo "$v $(grep '^{' gpurun_out/r04/pf2_one.log)" | tee -a gpurun_out/r04/pf2.log | cut -c1-100
  done
done
