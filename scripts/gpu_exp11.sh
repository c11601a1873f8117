#!/bin/bash
# light rows reading their workgroup's shared B rows from LDS (GCNK_LIGHT_HOT): time, forward, parity
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
PROBE=scripts/hub_probe.py bash scripts/variant_prof.sh "--reps 100 --variants row --widths 200" base hot base hot || exit 3
for R in 1 2; do for V in base hot; do
  if [ $V = base ]; then unset GCNK_LIB; else export GCNK_LIB=$PWD/_variants/libgcnk_$V.so; fi
  echo "$V $R $(timeout -k 10 200 python3 scripts/fuse_probe.py 2>&1 | grep '^{' | grep true | grep r8)"
done; done
unset GCNK_LIB
bash scripts/variants.sh hot; rc=$?; head -2 gpurun_out/var.log; exit $rc
