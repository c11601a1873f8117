cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/e4
for V in base rsc1; do
  if [ $V = base ]; then unset GCNK_LIB; else export GCNK_LIB=$PWD/_variants/libgcnk_$V.so; fi
  echo "== $V"; timeout -k 10 200 python3 scripts/fuse_probe.py 2>&1 | grep "^{" | grep true || exit 4
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/e4/tr_$V -o fwd -- python3 scripts/fwd_trace.py > gpurun_out/e4/tr_$V.log 2>&1 || exit 5
  python3 scripts/fwd_trace.py --report gpurun_out/e4/tr_$V | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['forward_span_us_median'], [k['us'] for k in d['kernels']])"
done
PROBE=scripts/hub_probe.py bash scripts/variant_prof.sh "--reps 100 --variants row --widths 200,8" base rsc1
