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
NS_ONLY=copy timeout -k 5 60 scripts/micro/ns_micro /tmp/r8.bin 128 > gpurun_out/micro/ns_copy.log 2>&1; echo "copy micro rc=$?"
grep variant gpurun_out/micro/ns_copy.log | cut -c1-160
timeout -k 10 300 python -u scripts/hub_probe.py --variants row --widths 200 --ipc 4,6,8,10,12,16 --reps 200 > gpurun_out/r04/probe_ipc.log 2>&1; echo "ipc sweep rc=$?"
grep -o '"ipc": [0-9]*\|"warm_us": [0-9.]*\|"cold_us": [0-9.]*\|"max_err": [0-9.e-]*' gpurun_out/r04/probe_ipc.log | paste - - - - 
GCNK_LIB=_variants/libgcnk_rowsc1.so timeout -k 10 300 python -u scripts/hub_probe.py --variants row --widths 200 --reps 200 > gpurun_out/r04/probe_sc1.log 2>&1; echo "sc1 rc=$?"
grep -o '"warm_us": [0-9.]*\|"cold_us": [0-9.]*' gpurun_out/r04/probe_sc1.log | paste - -
NS_ONLY=heavy timeout -k 5 60 scripts/micro/ns_micro /tmp/r8.bin 128 > gpurun_out/micro/ns_heavy.log 2>&1; echo "heavy micro rc=$?"
grep variant gpurun_out/micro/ns_heavy.log | cut -c1-220
timeout -k 10 400 python -u bench.py > gpurun_out/r04/bench.log 2>&1; echo "bench rc=$?"
tail -c 2500 gpurun_out/r04/bench.log
