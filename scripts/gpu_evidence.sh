#!/bin/bash
# The round's evidence set with the shipped library, in phases that each fit one gpurun call:
#   bash scripts/gpu_evidence.sh TAG tests|bench|pmc1|pmc2|iter|c5cpu|c5cpu64|dist
# Outputs under gpurun_out/TAG/ (copied into profiles/ afterwards).  Every GPU step runs under
# its own time limit; the first failing step ends the phase.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1; PHASE=$2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
sha256sum bayesopt_smart_amd/libbo_amd.so > "$OUT/lib_sha256.txt"
step() {   # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "[$name] rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || [ "$name" = "gpu_tests" -a $rc -eq 1 ] || exit $rc
}
pmc() {    # pmc NAME CMD...: one rocprofv3 --pmc pass per counter group, kernel trace only
  local name=$1; shift
  local d="$R/$OUT/pmc_$name"; mkdir -p "$d"
  local i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
             "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
             "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
    i=$((i + 1))
    ( cd /tmp && TMPDIR=/tmp timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
        -d "$d/p$i" -o run -- "$@" > "$d/p$i.log" 2>&1 ); local rc=$?
    echo "[pmc $name pass $i] rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
}
stats() {  # stats NAME CMD...: rocprofv3 --kernel-trace --stats
  local name=$1; shift
  ( cd /tmp && TMPDIR=/tmp timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$R/$OUT/stats_$name" -o run -- "$@" > "$R/$OUT/stats_$name.log" 2>&1 ); local rc=$?
  echo "[stats $name] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
B="python3 $R/bench.py"
case $PHASE in
  tests)
    step gpu_tests 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
  bench)
    step bench_c3_default 600 python bench.py
    step bench_c2 300 python bench.py --config C2 --steps 20 --warmup 5
    step bench_c4 400 python bench.py --config C4 --steps 5 --warmup 2
    step bench_c5 400 python bench.py --config C5 --steps 3 --warmup 2 --no-cpu-baseline
    step bench_c5f64 400 python bench.py --config C5 --mode auto --steps 3 --warmup 2 --no-cpu-baseline
    step bench_c3_hvi 300 python bench.py --acq hvi --steps 5 --warmup 2 --no-cpu-baseline
    step bench_c1 300 python bench.py --config C1 ;;
  pmc1)
    pmc c3 $B --steps 1 --warmup 1 --no-cpu-baseline
    pmc c2 $B --config C2 --steps 1 --warmup 1 --no-cpu-baseline
    pmc c4 $B --config C4 --steps 1 --warmup 1 --no-cpu-baseline
    stats c3 $B --steps 10 --warmup 3 --no-cpu-baseline
    stats c2 $B --config C2 --steps 20 --warmup 5 --no-cpu-baseline ;;
  pmc2)
    pmc c5 $B --config C5 --steps 1 --warmup 1 --no-cpu-baseline
    pmc c5f64 $B --config C5 --mode auto --steps 1 --warmup 1 --no-cpu-baseline ;;
  iter)
    step fit_c3 300 python bench.py --fit --config C3
    step fit_c4 300 python bench.py --fit --config C4
    step fit_c5 300 python bench.py --fit --config C5
    step iter_c3 500 python bench.py --iteration --config C3
    step iter_c5 500 python bench.py --iteration --config C5
    pmc fit $B --fit --config C3
    stats fit $B --fit --config C3 ;;
  c5cpu)      # C5 (fp32, the config's stated precision) with cpu_baseline and the whole set scored on
              # the host cores for selection_matches_cpu (--cpu-full: 4,194,304 candidates at N = 2048)
    step bench_c5_cpufull 1100 python -u bench.py --config C5 --steps 3 --warmup 2 --cpu-full ;;
  c5cpu64)
    step bench_c5f64_cpufull 1100 python -u bench.py --config C5 --mode auto --steps 3 --warmup 2 --cpu-full ;;
  dist)       # bench.py's multi-rank step rehearsed on one device (gloo, P = 1, 2, 4), C2 C3 C4 C5
    CFGS="C2 C3 C4 C5" step dist_rehearsal 1100 bash scripts/gpu_dist_rehearsal.sh
    cp gpurun_out/dist/rehearsal.jsonl "$OUT/dist_rehearsal.jsonl" ;;
  *) echo "unknown phase $PHASE"; exit 2 ;;
esac
