#!/bin/bash
# R8 training step: wall times (eager / graph / oracle) and a rocprofv3 kernel
# breakdown of the step (eager + graph replay).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 200 python -u scripts/bench_train.py --steps 50 --cpu-steps 3 > gpurun_out/r04/train.log 2>&1 || { echo "train rc=$?"; tail -5 gpurun_out/r04/train.log; exit 3; }
grep "^{" gpurun_out/r04/train.log
rm -rf gpurun_out/r04/train_trace
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04/train_trace -o tr -- python3 scripts/train_trace.py > gpurun_out/r04/train_trace.log 2>&1 || { echo "trace rc=$?"; tail -5 gpurun_out/r04/train_trace.log; exit 4; }
python scripts/train_trace.py --report gpurun_out/r04/train_trace > gpurun_out/r04/train_breakdown.json
head -c 2500 gpurun_out/r04/train_breakdown.json
find gpurun_out/r04/train_trace -name "*kernel_trace.csv" -delete
