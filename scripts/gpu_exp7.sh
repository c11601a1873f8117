#!/bin/bash
# forward timelines (rocprofv3 kernel trace) and forward times, base vs pair, twice
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
for R in 1 2; do for V in base pair; do
  if [ $V = base ]; then unset GCNK_LIB; else export GCNK_LIB=$PWD/_variants/libgcnk_$V.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/e7/tr_${V}_$R -o fwd -- python3 scripts/fwd_trace.py > gpurun_out/e7_$V.log 2>&1 || exit 5
  echo "$V $R $(python3 scripts/fwd_trace.py --report gpurun_out/e7/tr_${V}_$R | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['forward_span_us_median'], [k['us'] for k in d['kernels']])")"
  echo "$V $R $(timeout -k 10 200 python3 scripts/fuse_probe.py 2>&1 | grep '^{' | grep true | grep r8)"
done; done
