#!/bin/bash
# round 4: R8 / 20ng eval forward, factored vs SpMM path (record, hipGraph, HIP events)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
for f in 1 0 1 0; do
  GCNK_FACTOR_GC1=$f timeout -k 10 200 python -u scripts/factor_probe.py > gpurun_out/r04/fwd_path_$f.log 2>&1 || { echo "rc=$?"; exit 4; }
  grep "forward" gpurun_out/r04/fwd_path_$f.log | sed "s/^/factor=$f /"
done
