#!/bin/bash
# round 4: skinny GEMM (gc2's H1 W2) with its B values loaded ahead of the MFMAs; short-K GEMM scaling in M
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
rm -f gpurun_out/r04/skinny.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -p no:cacheprovider -x -q --timeout 120 --timeout-method thread -k "gemm or record or factored or trained" > gpurun_out/r04/pytest_27.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r04/pytest_27.log
[ $rc -eq 0 ] || exit $rc
for v in old product old product; do
  lib=""; [ $v != product ] && lib="GCNK_LIB=$PWD/_variants/libgcnk_$v.so"
  for shape in "18846 20 200" "7724 8 200" "1000 200 100" "4000 200 100" "18846 200 100"; do
    env $lib timeout -k 10 100 python -u scripts/gemm_probe.py $shape > gpurun_out/r04/sk_one.log 2>&1 || exit 4
    echo "$v $(grep '^{' gpurun_out/r04/sk_one.log)" | tee -a gpurun_out/r04/skinny.log | cut -c1-90
  done
done
