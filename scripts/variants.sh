#!/bin/bash
# Experiment driver (GPU box): for each prebuilt _variants/libgcnk_<name>.so,
# run the SpMM parity tests with it and time the sweep cases.
# usage: bash scripts/variants.sh name1 name2 ...   (SWEEP_ARGS to override)
set -o pipefail
mkdir -p gpurun_out
PKG=graph-convolutional-networks-for-text-classification_amd
for V in "$@"; do
  cp _variants/libgcnk_$V.so $PKG/libgcnk.so || exit 2
  echo "== $V" >> gpurun_out/var.log
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_$V.log 2>&1 || { tail -30 gpurun_out/pytest_$V.log; exit 3; }
  tail -1 gpurun_out/pytest_$V.log >> gpurun_out/var.log
  timeout -k 10 200 python scripts/sweep_spmm.py ${SWEEP_ARGS:---ipcs 16 --lanes 0} 2>/dev/null | grep -v hipSPARSE >> gpurun_out/var.log || exit 4
done
