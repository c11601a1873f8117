#!/bin/bash
# Hub plan group kernel ablations (rocprof kernel averages, cold rotation).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
bash scripts/variant_prof.sh "--variants hub --widths 200 --reps 200 --mode cold" base nostore nolight nocomp nocompstore
