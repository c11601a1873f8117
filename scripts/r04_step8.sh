#!/bin/bash
# round 4: NT row stores default, bwd2 reverted (+ H1 hoist), hub_xw batched hand-off loads
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 200 python -u scripts/factor_probe.py > gpurun_out/r04/factor_probe3.log 2>&1; echo "probe rc=$?"
grep "^{" gpurun_out/r04/factor_probe3.log
GCNK_FACTOR_XHUB=spmm timeout -k 10 200 python -u scripts/factor_probe.py --graphs r8 > gpurun_out/r04/factor_probe3s.log 2>&1; echo "probe spmm rc=$?"
grep "forward" gpurun_out/r04/factor_probe3s.log
timeout -k 10 300 python -u scripts/eager_fwd_profile.py > gpurun_out/r04/eager3.log 2>&1; echo "eager rc=$?"
grep -E "eager" gpurun_out/r04/eager3.log
timeout -k 10 300 python -u scripts/hub_probe.py --variants row,light,topic,copy --widths 200,8 --reps 200 > gpurun_out/r04/probe_nt_default.log 2>&1; echo "probe rc=$?"
grep "^{" gpurun_out/r04/probe_nt_default.log | cut -c1-330
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -p no:cacheprovider -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_d.log 2>&1; echo "pytest rc=$?"
tail -3 gpurun_out/r04/pytest_d.log
