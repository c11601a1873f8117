#!/bin/bash
# round 4: the 20ng-shaped forward on the SpMM path with gc2's projection fused (P = 20) or not
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
for p in 8 32 8 32; do
  GCNK_FACTOR_GC1=0 GCNK_FUSE_MAX_P=$p timeout -k 10 200 python -u scripts/factor_probe.py --graphs 20ng > gpurun_out/r04/fuse20_$p.log 2>&1 || { echo "rc=$?"; exit 4; }
  grep "forward" gpurun_out/r04/fuse20_$p.log | sed "s/^/fuse_max_p=$p /"
done
