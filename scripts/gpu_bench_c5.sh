cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py --config5 --cpu-sample-s 2 > gpurun_out/bench_c5.log 2>&1; rc=$?
tail -1 gpurun_out/bench_c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({k: d[k] for k in ('value','ms_per_step','roofline','config5_column_sharded')}, indent=1))"
exit $rc
