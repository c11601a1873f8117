#!/bin/bash
# tests + smoke + bench, then the rocprof kernel-trace summary of the bench
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
bash scripts/gpu_check.sh || exit $?
bash scripts/profile.sh
