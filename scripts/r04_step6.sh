#!/bin/bash
# round 4: why is each factored-forward kernel ~11 us in the bench trace?
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 200 python -u scripts/factor_probe.py > gpurun_out/r04/factor_probe.log 2>&1; echo "probe rc=$?"
grep "^{" gpurun_out/r04/factor_probe.log
GCNK_LIB=$PWD/_variants/libgcnk_oldfactor.so timeout -k 10 200 python -u scripts/factor_probe.py > gpurun_out/r04/factor_probe_old.log 2>&1; echo "probe old rc=$?"
grep "^{" gpurun_out/r04/factor_probe_old.log
GCNK_FACTOR_XHUB=spmm timeout -k 10 200 python -u scripts/factor_probe.py --graphs r8 > gpurun_out/r04/factor_probe_spmm.log 2>&1; echo "probe spmm rc=$?"
grep "^{" gpurun_out/r04/factor_probe_spmm.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04/fp_prof -o fp -- python3 scripts/factor_probe.py --graphs r8 > gpurun_out/r04/fp_prof.log 2>&1; echo "prof rc=$?"
find gpurun_out/r04/fp_prof -name "*kernel_stats.csv" -exec cut -d, -f1-8 {} \; | cut -c1-200
GCNK_LIB=$PWD/_variants/libgcnk_stamps.so timeout -k 10 120 python -u scripts/factor_stamps.py > gpurun_out/r04/factorstamps.log 2>&1; echo "factorstamps rc=$?"
tail -5 gpurun_out/r04/factorstamps.log | cut -c1-1500
