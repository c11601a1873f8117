#!/bin/bash
# One parameterised GPU-box driver (round 5 on; replaces the per-step rNN_stepK.sh
# scripts): every step runs under its own time limit, output goes to
# gpurun_out/<tag>/, and the first failing step ends the call.
#
# usage: scripts/gpu_run.sh <tag> <step> [<step> ...]
#   micro:<binary>[:<args>]   prebuilt scripts/micro/<binary> on the R8 A-hat (NS_ONLY, PROF honoured)
#   test:<pytest -k expr>     GPU tests matching the expression (-m gpu)
#   tests                     the whole GPU suite
#   bench[:<args>]            python bench.py <args> (default --steps 200 --warmup 20) -> bench.json
#   benchn:<name>:<args>      python bench.py <args> -> bench_<name>.json
#   prof:<script>[:<args>]    rocprofv3 --kernel-trace --stats over python scripts/<script> -> <script>_stats/
#   py:<script>[:<args>]      python scripts/<script> <args> -> <script>.log
#   vpy:<variant>:<script>[:<args>]  the same on _variants/libgcnk_<variant>.so
#   env:<NAME>=<value>        export for the following steps (env:<NAME>= unsets)
#   pmc:<c1,c2,..>:<script>[:<args>]  one rocprofv3 --pmc pass (counters comma-separated,
#                             within one pass's slots) over python scripts/<script> -> pmc<n>/
# prof/py/vpy outputs carry the step number (several runs of one script per call)
# Steps' outputs are summarised in profiles/ by hand (profiles/INDEX.md).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
tag="$1"; shift
out="gpurun_out/$tag"
mkdir -p "$out"
n=0
for step in "$@"; do
  n=$((n + 1))
  kind="${step%%:*}"; rest="${step#*:}"; [ "$rest" = "$step" ] && rest=""
  echo "=== $step" | tee -a "$out/steps.log"
  case "$kind" in
    micro)
      bin="${rest%%:*}"; args="${rest#*:}"; [ "$args" = "$rest" ] && args=""
      python3 scripts/micro/dump_r8.py /tmp/r8_adj.bin > /dev/null || exit 1
      timeout -k 10 240 "scripts/micro/$bin" /tmp/r8_adj.bin $args > "$out/$bin.log" 2>&1
      rc=$?; tail -n 80 "$out/$bin.log"; [ $rc -eq 0 ] || { echo "rc=$rc"; exit 1; }
      if [ -n "$PROF" ]; then
        timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/${bin}_prof" -o kt -- \
          "scripts/micro/$bin" /tmp/r8_adj.bin $args > "$out/${bin}_prof.log" 2>&1 || { echo "prof rc=$?"; exit 1; }
      fi ;;
    test)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$rest" \
        > "$out/pytest_$(echo "$rest" | tr -c 'A-Za-z0-9_' '_' | cut -c1-40).log" 2>&1
      rc=$?; tail -n 25 "$out"/pytest_*.log | tail -n 25; [ $rc -eq 0 ] || { echo "rc=$rc"; exit 1; } ;;
    tests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > "$out/pytest_gpu.log" 2>&1
      rc=$?; tail -n 15 "$out/pytest_gpu.log"; [ $rc -eq 0 ] || { echo "rc=$rc"; exit 1; } ;;
    bench)
      args="${rest:---steps 200 --warmup 20}"
      timeout -k 10 900 python -u bench.py $args --rocprof-dir "$out/bench_prof" > "$out/bench.json" 2> "$out/bench.err"
      rc=$?; tail -c 3000 "$out/bench.json"; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -n 20 "$out/bench.err"; exit 1; } ;;
    benchn)   # benchn:<name>:<args>: python bench.py <args> -> bench_<name>.json (several per call)
      nm="${rest%%:*}"; args="${rest#*:}"
      timeout -k 10 600 python -u bench.py $args > "$out/bench_$nm.json" 2> "$out/bench_$nm.err"
      rc=$?; tail -c 600 "$out/bench_$nm.json"; echo; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -n 20 "$out/bench_$nm.err"; exit 1; } ;;
    prof)
      s="${rest%%:*}"; args="${rest#*:}"; [ "$args" = "$rest" ] && args=""
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/${s%.py}_stats$n" -o kt -- \
        python3 "scripts/$s" $args > "$out/${s%.py}_prof$n.log" 2>&1
      rc=$?; tail -n 30 "$out/${s%.py}_prof$n.log"; [ $rc -eq 0 ] || { echo "rc=$rc"; exit 1; }
      python3 - "$out/${s%.py}_stats$n" <<'PY'
import csv, glob, sys
for f in glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"  {r['Name'][:100]:100s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:8.2f} us")
PY
      ;;
    py)
      s="${rest%%:*}"; args="${rest#*:}"; [ "$args" = "$rest" ] && args=""
      timeout -k 10 600 python3 -u "scripts/$s" $args > "$out/${s%.py}$n.log" 2>&1
      rc=$?; tail -n 60 "$out/${s%.py}$n.log"; [ $rc -eq 0 ] || { echo "rc=$rc"; exit 1; } ;;
    vpy)   # vpy:<variant name>:<script>[:<args>]: the script on _variants/libgcnk_<variant>.so
      v="${rest%%:*}"; rest2="${rest#*:}"
      s="${rest2%%:*}"; args="${rest2#*:}"; [ "$args" = "$rest2" ] && args=""
      GCNK_LIB="_variants/libgcnk_$v.so" timeout -k 10 600 python3 -u "scripts/$s" $args > "$out/${s%.py}_$v$n.log" 2>&1
      rc=$?; tail -n 60 "$out/${s%.py}_$v$n.log"; [ $rc -eq 0 ] || { echo "rc=$rc"; exit 1; } ;;
    pmc)
      ctrs="${rest%%:*}"; rest2="${rest#*:}"
      s="${rest2%%:*}"; args="${rest2#*:}"; [ "$args" = "$rest2" ] && args=""
      timeout -s KILL 120 rocprofv3 --pmc ${ctrs//,/ } --output-format csv -d "$out/pmc$n" -o pmc -- \
        python3 "scripts/$s" $args > "$out/pmc$n.log" 2>&1
      rc=$?; tail -n 5 "$out/pmc$n.log"; [ $rc -eq 0 ] || { echo "rc=$rc"; exit 1; } ;;
    env)
      name="${rest%%=*}"; val="${rest#*=}"
      if [ -n "$val" ]; then export "$name=$val"; else unset "$name"; fi ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "=== all steps done"
