#!/bin/bash
# round 4: gcn_bwd2 timeline after hoisting W2 and batching the partial-phase LDS reads; parity
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -p no:cacheprovider -x -q --timeout 120 --timeout-method thread -k "bwd2 or record or train" > gpurun_out/r04/pytest_17.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/r04/pytest_17.log
GCNK_LIB=$PWD/_variants/libgcnk_stamps.so timeout -k 10 120 python -u scripts/bwd2_stamps.py > gpurun_out/r04/bwd2_stamps2.log 2>&1; echo "stamps rc=$?"
grep "^{" gpurun_out/r04/bwd2_stamps2.log
timeout -k 10 300 python -u scripts/bench_train.py --steps 50 --cpu-steps 0 > gpurun_out/r04/train_17.log 2>&1; echo "train rc=$?"; grep "^{" gpurun_out/r04/train_17.log | cut -c1-200
for v in product bt512 bt1024; do
  lib=""; [ $v != product ] && lib="GCNK_LIB=$PWD/_variants/libgcnk_$v.so"
  env $lib timeout -k 10 120 python -u scripts/bwd2_probe.py > gpurun_out/r04/bwd2_probe_$v.log 2>&1; echo "$v rc=$?"; grep "^{" gpurun_out/r04/bwd2_probe_$v.log
done
