#!/bin/bash
# slab reduce with speculative slab loads (GCNK_REDUCE_SPEC): parity, op time, forward
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; exit $rc; }
PROBE=scripts/op_probe.py bash scripts/variant_prof.sh "--op XW1" base nospec base nospec || exit 3
for R in 1 2; do for V in base nospec; do
  if [ $V = base ]; then unset GCNK_LIB; else export GCNK_LIB=$PWD/_variants/libgcnk_$V.so; fi
  echo "$V $R $(timeout -k 10 200 python3 scripts/fuse_probe.py 2>&1 | grep '^{' | grep true | grep r8)"
done; done
