#!/bin/bash
# round 4: gc2's support H1 W2 at many rows through the short-K kernel (K <= 256, N <= 32) vs the skinny K-split kernel
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
rm -f gpurun_out/r04/narrow.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -p no:cacheprovider -x -q --timeout 120 --timeout-method thread -k "gemm or record or trained or config3 or factored" > gpurun_out/r04/pytest_30.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r04/pytest_30.log
[ $rc -eq 0 ] || exit $rc
for v in old product old product; do
  lib=""; [ $v != product ] && lib="GCNK_LIB=$PWD/_variants/libgcnk_$v.so"
  for shape in "18846 20 200" "7724 8 200" "18916 20 200" "4000 20 200"; do
    env $lib timeout -k 10 100 python -u scripts/gemm_probe.py $shape > gpurun_out/r04/nw_one.log 2>&1 || exit 4
    echo "$v $(grep '^{' gpurun_out/r04/nw_one.log)" | tee -a gpurun_out/r04/narrow.log | cut -c1-90
  done
  env $lib GCNK_FACTOR_GC1=0 timeout -k 10 200 python -u scripts/factor_probe.py --graphs 20ng > gpurun_out/r04/nw_fwd.log 2>&1 || exit 4
  echo "$v $(grep forward gpurun_out/r04/nw_fwd.log)" | tee -a gpurun_out/r04/narrow.log
done
