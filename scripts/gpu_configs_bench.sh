#!/bin/bash
# Bench lines for every BASELINE config on one GPU (C3 is the headline; the others are the
# per-config timings of DESIGN.md §6).  Stops at the first failing step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for c in ${CONFIGS:-C3 C2 C4 C5f64 C5}; do
  st=10; [ "$c" = C5 ] && st=3; [ "$c" = C4 ] && st=5
  args="--config $c"; [ "$c" = C5f64 ] && { args="--config C5 --mode auto"; st=3; }
  timeout -k 10 300 python -u bench.py $args --steps $st --warmup 2 ${BENCH_ARGS} > gpurun_out/bench_$c.log 2>&1; rc=$?
  echo "$c rc=$rc"; tail -1 gpurun_out/bench_$c.log
  [ $rc -eq 0 ] || exit $rc
done
