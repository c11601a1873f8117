#!/bin/bash
# A/B of prebuilt variants (_variants/libgcnk_<name>.so, "base" = in-tree):
# north-star op kernel times (rocprof) and the R8 / 20ng eval forward.
# usage: bash scripts/gpu_ab.sh name1 name2 ...
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
PROBE=scripts/hub_probe.py bash scripts/variant_prof.sh "--reps 100 --variants row --widths 200,8" "$@" || exit 3
for V in "$@"; do
  if [ $V = base ]; then unset GCNK_LIB; else export GCNK_LIB=$PWD/_variants/libgcnk_$V.so; fi
  echo "== forward $V"; timeout -k 10 200 python3 scripts/fuse_probe.py 2>&1 | grep "^{" | grep true || exit 4
done
