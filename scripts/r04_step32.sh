#!/bin/bash
# round 4: short-K GEMM with a row-block loop per workgroup slot (B staged once, next A under the MFMAs)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
rm -f gpurun_out/r04/shortk_loop.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -p no:cacheprovider -x -q --timeout 120 --timeout-method thread -k "gemm or record or config3" > gpurun_out/r04/pytest_32.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r04/pytest_32.log
[ $rc -eq 0 ] || exit $rc
for v in noloop product w1024 w256 noloop product; do
  lib=""; [ $v != product ] && lib="GCNK_LIB=$PWD/_variants/libgcnk_$v.so"
  for shape in "18846 200 100" "70 200 100" "18846 20 200"; do
    env $lib timeout -k 10 100 python -u scripts/gemm_probe.py $shape > gpurun_out/r04/sl_one.log 2>&1 || exit 4
    echo "$v $(grep '^{' gpurun_out/r04/sl_one.log)" | tee -a gpurun_out/r04/shortk_loop.log | cut -c1-90
  done
  env $lib timeout -k 10 200 python -u scripts/factor_probe.py --graphs 20ng > gpurun_out/r04/sl_fwd.log 2>&1 || exit 4
  echo "$v $(grep forward gpurun_out/r04/sl_fwd.log)" | tee -a gpurun_out/r04/shortk_loop.log
done
