#!/bin/bash
# round 4: short-K GEMM column tile width (GCNK_SHORTK_NT 7 / 5 / 4 / 3 n16-tiles per workgroup)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
rm -f gpurun_out/r04/shortk_nt.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -p no:cacheprovider -x -q --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/r04/pytest_28.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/r04/pytest_28.log; exit 3; }
for v in ${VARIANTS:-product nt5 nt4 nt3 product nt4 nt3}; do
  lib=""; [ $v != product ] && lib="GCNK_LIB=$PWD/_variants/libgcnk_$v.so"
  for shape in "70 200 100" "1000 200 100" "18846 200 100" "18916 200 100"; do
    env $lib timeout -k 10 100 python -u scripts/gemm_probe.py $shape > gpurun_out/r04/sk_one.log 2>&1 || exit 4
    echo "$v $(grep '^{' gpurun_out/r04/sk_one.log)" | tee -a gpurun_out/r04/shortk_nt.log | cut -c1-90
  done
done
