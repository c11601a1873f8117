#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r04 gpurun_out/micro
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/r04/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error|FAIL" gpurun_out/r04/pytest_gpu.log | tail -n 20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
python3 scripts/micro/dump_r8.py /tmp/r8.bin >/dev/null || exit 3
NS_ONLY=lds timeout -k 5 60 scripts/micro/ns_micro /tmp/r8.bin 128 > gpurun_out/micro/ns_lds.log 2>&1; echo "lds micro rc=$?"
grep variant gpurun_out/micro/ns_lds.log | cut -c1-220; tail -2 gpurun_out/micro/ns_lds.log | cut -c1-200
NS_ONLY=heavy timeout -k 5 60 scripts/micro/ns_micro /tmp/r8.bin 128 > gpurun_out/micro/ns_heavy.log 2>&1; echo "heavy micro rc=$?"
grep variant gpurun_out/micro/ns_heavy.log | cut -c1-220
timeout -k 10 400 python -u bench.py > gpurun_out/r04/bench.log 2>&1; echo "bench rc=$?"
tail -c 2500 gpurun_out/r04/bench.log
