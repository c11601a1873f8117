#!/bin/bash
# round 4: small-M split-K GEMM column tile (7 / 4 / 3 n16-tiles) for R8's X_hubs W1, against the tile plan
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
rm -f gpurun_out/r04/smallm_nt.log
for v in product sm4 sm3 product sm4 sm3; do
  lib=""; [ $v != product ] && lib="GCNK_LIB=$PWD/_variants/libgcnk_$v.so"
  for sp in 59 117 234; do
    env $lib GCNK_PROBE_SPLIT=$sp timeout -k 10 100 python -u scripts/gemm_probe.py 50 200 7464 > gpurun_out/r04/sm_one.log 2>&1 || exit 4
    echo "$v $(grep '^{' gpurun_out/r04/sm_one.log)" | tee -a gpurun_out/r04/smallm_nt.log | cut -c1-100
  done
  env $lib GCNK_FACTOR_XHUB=gemm timeout -k 10 200 python -u scripts/factor_probe.py --graphs r8 > gpurun_out/r04/sm_fwd.log 2>&1 || exit 4
  grep "X_hubs\|forward" gpurun_out/r04/sm_fwd.log | sed "s/^/$v /" | tee -a gpurun_out/r04/smallm_nt.log
done
