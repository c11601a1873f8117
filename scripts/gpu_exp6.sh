#!/bin/bash
# X W1 chunk pairing (GCNK_TILE_PAIR): timing, forward, HBM traffic, then the parity tests with it
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
PROBE=scripts/op_probe.py bash scripts/variant_prof.sh "--op XW1" base pair base pair || exit 3
for V in base pair; do
  if [ $V = base ]; then unset GCNK_LIB; else export GCNK_LIB=$PWD/_variants/libgcnk_$V.so; fi
  echo "== forward $V"; timeout -k 10 200 python3 scripts/fuse_probe.py 2>&1 | grep "^{" | grep true || exit 4
  D=gpurun_out/pmc_$V; mkdir -p $D
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- python3 scripts/pmc_ops.py --op XW1 > $D/fetch.log 2>&1 || exit 5
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- python3 scripts/pmc_ops.py --op XW1 > $D/write.log 2>&1 || exit 5
  python3 scripts/pmc_summary.py $D | python3 -c "import json,sys; d=json.load(sys.stdin); print({k: round(v.get('hbm_bytes_per_launch',0)/1e6,2) for k,v in d.items()})"
done
unset GCNK_LIB
bash scripts/variants.sh pair; rc=$?; cat gpurun_out/var.log | tail -3; exit $rc
