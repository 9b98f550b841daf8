#!/bin/bash
# A/B of library variants over several configs in one box: CONFIGS (default "C2 C3 C4"), each lib.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
LIBS=${LIBS:-$(ls bayesopt_smart_amd/libbo_amd*.so)}
: > gpurun_out/ab.jsonl
for c in ${CONFIGS:-C2 C3 C4}; do
  for lib in $LIBS; do
    BO_AMD_LIB=$R/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --config $c ${BENCH_ARGS} > gpurun_out/ab_one.json 2> gpurun_out/ab_err.log; rc=$?
    [ $rc -eq 0 ] || { echo "$c $lib rc=$rc"; tail -5 gpurun_out/ab_err.log; exit $rc; }
    python -c "import json; d=json.load(open('gpurun_out/ab_one.json')); d['lib']='$lib'; d['cfg']='$c'; print(json.dumps(d))" >> gpurun_out/ab.jsonl
    python -c "import json; d=json.load(open('gpurun_out/ab_one.json')); r=d['roofline']; print('$c', '$lib', round(d['ms_per_step'],3), round(r['kernel_ms'],3), round(r['frac'],3))"
  done
done
