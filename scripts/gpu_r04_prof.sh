#!/bin/bash
# Round-4 evidence, part C: rocprofv3 kernel stats and PMC summaries of the shipped library.
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out
TAG=${1:-r04_final}
stats() {   # stats NAME ARGS...: kernel-trace --stats of one bench command
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_st_$name -o run -- python3 $R/bench.py "$@") \
    > gpurun_out/${TAG}_st_$name.log 2>&1 || { echo "stats $name failed"; tail gpurun_out/${TAG}_st_$name.log; exit 1; }
  f=$(find gpurun_out/${TAG}_st_$name -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${TAG}_${name}_kernel_stats.csv
  echo "== $name"; cut -d, -f1-4 gpurun_out/${TAG}_${name}_kernel_stats.csv | head -4
}
pmc() {     # pmc NAME WORKLOAD ALG_BYTES KERNEL_FILTER ARGS...
  local name=$1 wl=$2 alg=$3 kf=$4; shift 4
  OUT=gpurun_out/${TAG}_pmc_$name bash scripts/pmc_run.sh python3 $R/bench.py "$@" || { echo "pmc $name failed"; exit 1; }
  PMC_KERNEL=$kf python3 scripts/pmc_summary.py gpurun_out/${TAG}_pmc_$name gpurun_out/${TAG}_${name}_pmc.json "$wl" "$alg" "$kf" > /dev/null \
    || { echo "pmc summary $name failed"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], {k: d.get(k) for k in ('hbm_bytes_per_launch','algorithmic_bytes_per_launch','traffic_ratio','non_mfma_valu_per_mfma','wait_inst_any_per_busy_cycle')})" gpurun_out/${TAG}_${name}_pmc.json
}
if [ "${SET:-1}" = "1" ]; then
  stats c3 --steps 20 --warmup 3 --no-cpu-baseline
  stats c2 --config C2 --steps 50 --warmup 5 --no-cpu-baseline
  stats fit --fit --config C3
  pmc c3 C3 41943040 predict_kernel --steps 2 --warmup 1 --no-cpu-baseline
  PMC_ALG_NOTE="56 B per candidate: mu, var, UCB of 2 objectives (6 x 8 B) + acq (8 B), as the C2 bench line" \
    pmc c2 C2 14680064 predict_kernel --config C2 --steps 2 --warmup 1 --no-cpu-baseline
  pmc fit "fit C3" none fit_persist_kernel --fit --config C3
else
  pmc c4 C4 218103808 predict_kernel --config C4 --steps 1 --warmup 1 --no-cpu-baseline
  pmc c5 C5 436207616 predict_kernel --config C5 --steps 1 --warmup 1 --no-cpu-baseline
  pmc c5f64 C5-auto 436207616 predict_kernel --config C5 --mode auto --steps 1 --warmup 1 --no-cpu-baseline
fi
