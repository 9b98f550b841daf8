#!/bin/bash
# rocprofv3 kernel stats of bench.py steps for several libraries (per-step kernels: prep, fused,
# merge), interleaved twice: gpu_prof_step.sh TAG "CFGS" "LIBS"
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; CFGS=${2:-"C2 C3"}; LIBS=${3:-bayesopt_smart_amd/libbo_amd.so}
export TMPDIR=/tmp
cd /tmp
for rnd in 1 2; do
  for c in $CFGS; do
    for lib in $LIBS; do
      n=$(basename $lib .so)
      d="$R/gpurun_out/profstep_${TAG}_${c}_${n}_$rnd"
      BO_AMD_LIB=$R/$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- \
          python3 "$R/bench.py" --config $c --steps 30 --warmup 3 --no-cpu-baseline > "$d.log" 2>&1 || { echo "fail $c $n"; tail -5 "$d.log"; exit 1; }
      f=$(find "$d" -name "*kernel_stats.csv" | head -1)
      echo "== $c $n $rnd $(python3 -c "import json,sys; l=[x for x in open('$d.log') if x.startswith('{')][-1]; d=json.loads(l); print(round(d['ms_per_step'],4), d['roofline']['kernel_ms'], d.get('selection_matches_cpu'))")"
      python3 -c "import csv; [print('  ', r['Name'].replace('(anonymous namespace)::','')[:40], r['Calls'], r['AverageNs'], r['MinNs']) for r in csv.DictReader(open('$f'))]"
    done
  done
done
