#!/bin/bash
# One GPU session of named steps, each under its own time limit; stops at the first step that
# crashes, aborts or times out (pytest's rc 1 = test failures is reported and the run goes on).
#   scripts/gpu_run.sh TAG step [step ...]
#   steps: tests[:<files>[|<-k expr, + for space>]]  smoke  bench[:<bench args>]  iter:<cfg>  fit:<cfg>
#          prof:<bench args>  (rocprofv3 --kernel-trace --stats of bench.py)
#          py:<script args>  pyprof:<script args> (rocprofv3 of a python script)
#          env:VAR=value (exported for the following steps; env:VAR= unsets it)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1; shift
mkdir -p gpurun_out
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
STEP_OK() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
i=0
for st in "$@"; do
  i=$((i + 1))
  kind=${st%%:*}; arg=""; [ "$kind" != "$st" ] && arg=${st#*:}
  case $kind in
    tests)
      # tests:FILES or tests:FILES|KEXPR (a -k expression, '+' for a space: tests:x.py|a+or+b)
      sel=${arg:-tests}; kx=""
      if [ "${sel#*|}" != "$sel" ]; then kx=${sel#*|}; kx=${kx//+/ }; sel=${sel%%|*}; fi
      if [ -n "$kx" ]; then
        timeout -k 10 1200 python -u -m pytest $sel -k "$kx" -m gpu -v --timeout 300 --timeout-method thread -rf \
            > "$OUT/tests_$i.log" 2>&1; rc=$?
      else
        timeout -k 10 1200 python -u -m pytest $sel -m gpu -v --timeout 300 --timeout-method thread -rf \
            > "$OUT/tests_$i.log" 2>&1; rc=$?
      fi
      echo "[$i] pytest $sel rc=$rc"; grep -E "passed|failed|error" "$OUT/tests_$i.log" | tail -3 ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
      echo "[$i] smoke rc=$rc"; tail -2 "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 600 python bench.py $arg > "$OUT/bench_$i.jsonl" 2> "$OUT/bench_$i.err"; rc=$?
      echo "[$i] bench $arg rc=$rc"; tail -c 1500 "$OUT/bench_$i.jsonl"; echo ;;
    iter)
      timeout -k 10 600 python bench.py --iteration --config $arg > "$OUT/iter_$arg.jsonl" 2> "$OUT/iter_$arg.err"; rc=$?
      echo "[$i] iteration $arg rc=$rc"; tail -c 2500 "$OUT/iter_$arg.jsonl"; echo ;;
    fit)
      timeout -k 10 300 python bench.py --fit --config $arg > "$OUT/fit_$arg.jsonl" 2> "$OUT/fit_$arg.err"; rc=$?
      echo "[$i] fit $arg rc=$rc"; tail -c 2500 "$OUT/fit_$arg.jsonl"; echo ;;
    prof)
      export TMPDIR=/tmp
      ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_$i" -o run -- \
          python "$R/bench.py" $arg > "$R/$OUT/prof_$i.log" 2>&1 ); rc=$?
      echo "[$i] rocprof $arg rc=$rc"; tail -2 "$OUT/prof_$i.log"
      f=$(find "$OUT/prof_$i" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -12 "$f" | cut -c1-200 ;;
    env)
      arg=${arg//@R@/$R}
      if [ -z "${arg#*=}" ]; then unset "${arg%%=*}"; else export "$arg"; fi
      echo "[$i] env $arg"; rc=0 ;;
    pyprof)
      export TMPDIR=/tmp
      ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/pyprof_$i" -o run -- \
          python $(cd "$R" && echo "$R/$arg") > "$R/$OUT/pyprof_$i.log" 2>&1 ); rc=$?
      echo "[$i] rocprof python $arg rc=$rc"; tail -3 "$OUT/pyprof_$i.log"
      f=$(find "$OUT/pyprof_$i" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -12 "$f" | cut -c1-200 ;;
    py)
      timeout -k 10 600 python $arg > "$OUT/py_$i.log" 2>&1; rc=$?
      echo "[$i] python $arg rc=$rc"; tail -20 "$OUT/py_$i.log" ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
  STEP_OK $rc || { echo "stopping after [$i] $st (rc=$rc)"; exit $rc; }
done
