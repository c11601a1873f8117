#!/bin/bash
# round 4: record parity tests + north-star (row kernel, heavy-gather fix) cold/warm + eager timing + micro
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "record or factored or gcn_ or trained or graph_capture or device_dropout or spmm_r8 or widths or schedule" \
  > gpurun_out/r04/pytest_a.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error|FAIL" gpurun_out/r04/pytest_a.log | tail -n 30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/hub_probe.py --variants row,copy --widths 200,8 --reps 200 > gpurun_out/r04/probe.log 2>&1 || { echo "probe failed"; tail gpurun_out/r04/probe.log; exit 3; }
cut -c1-400 gpurun_out/r04/probe.log
for v in hu8 hu16; do
  GCNK_LIB=_variants/libgcnk_$v.so timeout -k 10 300 python -u scripts/hub_probe.py --variants row --widths 200 --reps 200 > gpurun_out/r04/probe_$v.log 2>&1 || { echo "probe $v failed"; tail gpurun_out/r04/probe_$v.log; exit 3; }
  echo "$v: $(grep -o '"warm_us.*cold_frac[^,]*' gpurun_out/r04/probe_$v.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04/prof_cold -o kt -- python3 scripts/hub_probe.py --variants row --widths 200 --reps 200 --mode cold > gpurun_out/r04/prof_cold.log 2>&1 || { echo "rocprof failed"; tail gpurun_out/r04/prof_cold.log; exit 3; }
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r04/prof_cold/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "spmm" in r["Name"] or "elementwise" in r["Name"]:
            print(f"  {r['Name'][:90]:90s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:7.3f} us")
PY
timeout -k 10 300 python -u scripts/eager_fwd_profile.py > gpurun_out/r04/eager.log 2>&1
rc2=$?; echo "eager rc=$rc2"; head -n 8 gpurun_out/r04/eager.log
if [ $rc2 -ne 0 ]; then exit $rc2; fi
bash scripts/micro/run_ns_micro.sh 128 > /dev/null 2>&1; echo "micro rc=$?"
grep -E "variant" gpurun_out/micro/ns.log | cut -c1-200
