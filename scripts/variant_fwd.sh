#!/bin/bash
# Forward kernel timeline (scripts/fwd_trace.py under rocprofv3) for each
# experiment variant named on the command line ("base" = the product library),
# with the factored gc1 and, when FACTOR0=1, also with GCNK_FACTOR_GC1=0.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
for V in "$@"; do
  for F in 1 ${FACTOR0:+0}; do
    if [ "$V" = base ]; then unset GCNK_LIB; else export GCNK_LIB=$PWD/_variants/libgcnk_$V.so; fi
    export GCNK_FACTOR_GC1=$F
    rm -rf gpurun_out/vt/$V$F
    timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vt/$V$F -o fwd -- \
      python3 scripts/fwd_trace.py > gpurun_out/vt_$V$F.log 2>&1 || { echo "$V rc=$?"; exit 4; }
    echo "== $V factor=$F"
    python3 scripts/fwd_trace.py --report gpurun_out/vt/$V$F | grep -o '"us": [0-9.]*\|span_us_median": [0-9.]*' | tr '\n' ' '
    echo
  done
done
