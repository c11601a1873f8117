#!/bin/bash
# round 4: kernel split of the small-M split-K GEMM (rocprof) and the forward's kernel timeline
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
rm -rf gpurun_out/r04/smallm_prof
GCNK_PROBE_SPLIT=117 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04/smallm_prof -o p -- \
  python3 scripts/gemm_probe.py 50 200 7464 > gpurun_out/r04/smallm_prof.log 2>&1; echo "prof rc=$?"
f=$(find gpurun_out/r04/smallm_prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -8
bash scripts/variant_fwd.sh base
