#!/bin/bash
# Round-3 evidence in one GPU session (each step under its own time limit; stops at the first
# failure): GPU tests, smoke, PMC summaries of the fused kernel per config (stamped with the
# library's sha256, copied into profiles/ on the box so that bench.py's traffic field uses them),
# the per-config bench lines, the default C3 line, the exact-HVI line, the fit lines, rocprofv3
# kernel stats of C3, C2 and the C3 fit, and PMC of the fit kernels.  Everything lands under
# gpurun_out/ev/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
E=gpurun_out/ev
mkdir -p $E
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $E/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $E/gpu_tests.log; exit 1; }
tail -1 $E/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $E/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 $E/smoke.log
# PMC per config: one counter group per pass (kernel-trace only)
pmc() {   # name, workload key (bench.py's pmc_traffic), kernel filter, alg bytes, label, bench args...
  local name=$1 key=$2 filt=$3 alg=$4 label=$5; shift 5
  mkdir -p $R/$E/pmc_$name
  local i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
             "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
             "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
             "SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS"; do
    i=$((i+1))
    (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$R/$E/pmc_$name/p$i" -o run -- \
       python3 "$R/bench.py" "$@" > "$R/$E/pmc_$name/p$i.log" 2>&1) || { echo "pmc $name pass $i failed"; return 1; }
  done
  PMC_KERNEL=$filt python3 scripts/pmc_summary.py $E/pmc_$name $E/r03_final_${name}_pmc.json $key $alg "$label" > /dev/null || return 1
  cp $E/r03_final_${name}_pmc.json profiles/
  echo "pmc $name ok"
}
pmc c3 C3 cm_predict_kernel $((8*5*1048576)) "cm_predict_kernel<2, true, true, false, 16>" --config C3 --steps 1 --warmup 1 --no-cpu-baseline || exit 1
pmc c2 C2 cm_predict_kernel $((8*5*262144)) "cm_predict_kernel<2, true, true, false, 4>" --config C2 --steps 1 --warmup 1 --no-cpu-baseline || exit 1
pmc c4 C4 cm_predict_kernel $((8*(7+6)*2097152)) "cm_predict_kernel<6, false, true, false, 16>" --config C4 --steps 1 --warmup 1 --no-cpu-baseline || exit 1
pmc c5f64 C5-auto cm_predict_kernel $((8*(7+6)*4194304)) "cm_predict_kernel<6, false, true, true, 16>" --config C5 --mode auto --steps 1 --warmup 1 --no-cpu-baseline || exit 1
pmc c5 C5 cm32_predict_kernel $((8*(7+6)*4194304)) "cm32_predict_kernel<6>" --config C5 --steps 1 --warmup 1 --no-cpu-baseline || exit 1
pmc fit FIT-C3 fit_step_kernel 1 "fit_step_kernel (compute_mll / invert_k steps, C3 N = 512)" --fit --config C3 || exit 1
# bench lines (the PMC summaries above are now in profiles/ with this library's sha)
for c in C3 C2 C4 C5f64 C5; do
  st=10; [ "$c" = C5 ] && st=3; [ "$c" = C4 ] && st=5
  args="--config $c"; [ "$c" = C5f64 ] && { args="--config C5 --mode auto"; st=3; }
  timeout -k 10 400 python -u bench.py $args --steps $st --warmup 2 > $E/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -5 $E/bench_$c.log; exit 1; }
  tail -1 $E/bench_$c.log >> $E/configs_bench.jsonl
done
echo configs ok
timeout -k 10 400 python -u bench.py > $E/default_bench.jsonl 2> $E/default_bench.err || { echo "default bench failed"; exit 1; }
timeout -k 10 400 python -u bench.py --acq hvi > $E/hvi_bench.jsonl 2> $E/hvi_bench.err || { echo "hvi bench failed"; exit 1; }
: > $E/fit.jsonl
for c in C3 C4 C5; do
  timeout -k 10 400 python -u bench.py --fit --config $c >> $E/fit.jsonl 2>> $E/fit.err || { echo "fit $c failed"; exit 1; }
done
timeout -k 10 300 python -u scripts/select_ubench.py > $E/select_ubench.jsonl 2>&1 || { echo "select ubench failed"; exit 1; }
echo benches ok
for c in C3 C2; do
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$E/prof_$c" -o run -- \
      python3 "$R/bench.py" --config $c --steps 5 --warmup 2 --no-cpu-baseline > "$R/$E/prof_$c.log" 2>&1) || { echo "prof $c failed"; exit 1; }
done
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$E/prof_fit" -o run -- \
    python3 "$R/bench.py" --fit --config C3 > "$R/$E/prof_fit.log" 2>&1) || { echo "prof fit failed"; exit 1; }
echo done
