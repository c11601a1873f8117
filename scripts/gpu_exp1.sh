cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
bash scripts/variant_prof.sh "--reps 100 --variants row --widths 200,8" base pf hv hvpf || exit 3
timeout -k 10 200 python3 scripts/fuse_probe.py > gpurun_out/fuse_probe.log 2>&1; rc=$?; grep "^{" gpurun_out/fuse_probe.log; exit $rc
