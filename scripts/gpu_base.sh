cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
bash scripts/gpu_check.sh || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fwdtr -o fwd -- python3 scripts/fwd_trace.py > gpurun_out/fwdtr.log 2>&1 || { echo "trace rc=$?"; exit 3; }
python3 scripts/fwd_trace.py --report gpurun_out/fwdtr > gpurun_out/fwdtr_report.json
cat gpurun_out/fwdtr_report.json
