#!/bin/bash
# skinny GEMM with 64-row workgroups (GCNK_SKINNY_RT): parity, 20ng timings
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; exit $rc; }
PROBE=scripts/fwd20_probe.py bash scripts/variant_prof.sh "" base rt1 base rt1 || exit 3
