#!/bin/bash
# Round-2 final evidence: GPU tests, bench line (with the rocprof summaries the
# roofline comes from), rocprofv3 kernel stats of a bench run (forward graphs),
# and the forward's per-kernel timeline.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r02f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest rc=$?"; tail -5 $O/pytest_gpu.log; exit 3; }
tail -1 $O/pytest_gpu.log
timeout -k 10 500 python3 bench.py --rocprof-dir $O/bench_rocprof > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/bench.log; exit 3; }
tail -1 $O/bench.log > $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fwd -o fwd -- \
  python3 bench.py --steps 200 --warmup 20 --no-pmc --cpu-sample-s 0 --no-configs --no-rocprof --kernel-reps 1 > $O/prof_fwd.log 2>&1 \
  || { echo "prof fwd rc=$?"; exit 3; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/fwdtr -o fwd -- python3 scripts/fwd_trace.py > $O/fwdtr.log 2>&1 \
  || { echo "trace rc=$?"; exit 3; }
python3 scripts/fwd_trace.py --report $O/fwdtr > $O/fwdtr_report.json
echo done
