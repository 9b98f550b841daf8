#!/bin/bash
# rocprofv3 kernel-trace summaries of bench.py per config: prof_cfg.sh TAG CONFIG [CONFIG ...]
# -> gpurun_out/prof_<TAG>_<CONFIG>/ (stats CSVs) and .log
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
export TMPDIR=/tmp
cd /tmp
for c in "$@"; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}_$c" -o run -- \
      python "$R/bench.py" --config "$c" --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > "$R/gpurun_out/prof_${TAG}_$c.log" 2>&1
  rc=$?
  echo "prof $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  f=$(find "$R/gpurun_out/prof_${TAG}_$c" -name "*kernel_stats.csv" | head -1)
  cut -d, -f1-4 "$f" | head -8
done
