#!/bin/bash
# round 4: counters on their own lines (hub_xw, gcn_bwd2), round-3 hubfactor restored; 20ng hubfactor timeline
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 200 python -u scripts/factor_probe.py > gpurun_out/r04/factor_probe2.log 2>&1; echo "probe rc=$?"
grep "^{" gpurun_out/r04/factor_probe2.log
GCNK_STAMP_GRAPH=20ng GCNK_LIB=$PWD/_variants/libgcnk_stamps.so timeout -k 10 120 python -u scripts/factor_stamps.py > gpurun_out/r04/factorstamps20.log 2>&1; echo "factorstamps20 rc=$?"
grep "^{" gpurun_out/r04/factorstamps20.log | cut -c1-1500
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -p no:cacheprovider -x -q --timeout 120 --timeout-method thread \
  -k "bwd2 or hub_xw or factor or record or trained" > gpurun_out/r04/pytest_c.log 2>&1; echo "pytest rc=$?"
tail -3 gpurun_out/r04/pytest_c.log
timeout -k 10 300 python -u scripts/eager_fwd_profile.py > gpurun_out/r04/eager2.log 2>&1; echo "eager rc=$?"
grep -E "eager" gpurun_out/r04/eager2.log
timeout -k 10 300 python -u scripts/hub_probe.py --variants row,copy --widths 200 --reps 200 > gpurun_out/r04/probe_prod.log 2>&1; echo "prod rc=$?"
grep "^{" gpurun_out/r04/probe_prod.log | cut -c1-250
GCNK_LIB=$PWD/_variants/libgcnk_rownt.so timeout -k 10 300 python -u scripts/hub_probe.py --variants row,light,topic --widths 200 --reps 200 > gpurun_out/r04/probe_nt.log 2>&1; echo "nt rc=$?"
grep "^{" gpurun_out/r04/probe_nt.log | cut -c1-250
