#!/bin/bash
# chunk pairing with the second chunk's loads under the first's MFMAs: op time, forward timelines, parity
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
PROBE=scripts/op_probe.py bash scripts/variant_prof.sh "--op XW1" base pair || exit 3
bash scripts/gpu_exp7.sh || exit 4
unset GCNK_LIB
bash scripts/variants.sh pair; rc=$?; head -2 gpurun_out/var.log; exit $rc
