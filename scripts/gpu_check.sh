#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Stops at the first step that crashes/aborts/times out (exit >= 2 other than pytest's 1).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
STEP_OK() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -rf ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -25 gpurun_out/gpu_tests.log
  STEP_OK $rc || exit $rc
fi
if [ "$MODE" = all ] || [ "$MODE" = smoke ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
  STEP_OK $rc || exit $rc
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
  STEP_OK $rc || exit $rc
fi
if [ "$MODE" = all ] || [ "$MODE" = fit ]; then
  : > gpurun_out/fit.jsonl
  for c in C3 C4 C5; do
    timeout -k 10 300 python bench.py --fit --config $c >> gpurun_out/fit.jsonl 2> gpurun_out/fit_$c.err; rc=$?
    echo "fit $c rc=$rc"; tail -c 600 gpurun_out/fit.jsonl; echo
    STEP_OK $rc || exit $rc
  done
fi
if [ "$MODE" = configs ]; then
  : > gpurun_out/configs.jsonl
  for c in C2 C3 C4 C5; do
    timeout -k 10 300 python bench.py --config $c >> gpurun_out/configs.jsonl 2> gpurun_out/cfg_$c.err; rc=$?
    echo "config $c rc=$rc"
    STEP_OK $rc || exit $rc
  done
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  export TMPDIR=/tmp
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- \
      python "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > "$R/gpurun_out/prof.log" 2>&1; rc=$?
  echo "rocprof rc=$rc"; tail -3 "$R/gpurun_out/prof.log"
  find "$R/gpurun_out/prof" -name "*stats*" | head
fi
