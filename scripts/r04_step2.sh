#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/eager_fwd_profile.py > gpurun_out/r04/eager.log 2>&1
rc2=$?; echo "eager rc=$rc2"; head -n 30 gpurun_out/r04/eager.log
if [ $rc2 -ne 0 ]; then exit $rc2; fi
bash scripts/micro/run_ns_micro.sh 128 > /dev/null 2>&1; echo "micro rc=$?"
grep -E "variant" gpurun_out/micro/ns.log | cut -c1-200
