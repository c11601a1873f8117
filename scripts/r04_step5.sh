#!/bin/bash
# round 4: full GPU suite, store-policy micro, sc1 row variant, bench, eager step
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r04 gpurun_out/micro
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -p no:cacheprovider -x -q -s --timeout 120 --timeout-method thread \
  > gpurun_out/r04/pytest_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|trained model|FAIL|Error" gpurun_out/r04/pytest_full.log | tail -n 12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
python3 scripts/micro/dump_r8.py /tmp/r8.bin >/dev/null || exit 3
for v in copy lds; do
  NS_ONLY=$v timeout -k 5 90 scripts/micro/ns_micro /tmp/r8.bin 128 > gpurun_out/micro/ns_$v.log 2>&1; echo "$v micro rc=$?"
  grep -E "variant|hipFunc|error" gpurun_out/micro/ns_$v.log | cut -c1-240
done
timeout -k 10 300 python -u scripts/hub_probe.py --variants row,light,topic,copy --widths 200,8 --reps 200 > gpurun_out/r04/probe_subsets.log 2>&1; echo "subsets rc=$?"
cut -c1-300 gpurun_out/r04/probe_subsets.log | grep -v amdgpu.ids
GCNK_LIB=_variants/libgcnk_rowsc1.so timeout -k 10 300 python -u scripts/hub_probe.py --variants row,light,topic,copy --widths 200 --reps 200 > gpurun_out/r04/probe_sc1.log 2>&1; echo "sc1 rc=$?"
cut -c1-300 gpurun_out/r04/probe_sc1.log | grep -v amdgpu.ids
timeout -k 10 500 python -u bench.py > gpurun_out/r04/bench.log 2>&1; echo "bench rc=$?"
tail -c 600 gpurun_out/r04/bench.log
timeout -k 10 300 python -u scripts/eager_fwd_profile.py > gpurun_out/r04/eager.log 2>&1; echo "eager rc=$?"
grep -E "eager" gpurun_out/r04/eager.log
