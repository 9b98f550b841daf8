#!/bin/bash
# A/B of library variants on one config: BENCH_ARGS, then each lib in LIBS (default: the
# product library and every diagnostic build present).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
LIBS=${LIBS:-$(ls bayesopt_smart_amd/libbo_amd*.so)}
: > gpurun_out/ab.jsonl
for lib in $LIBS; do
  BO_AMD_LIB=$R/$lib timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab_one.json 2> gpurun_out/ab_err.log; rc=$?
  echo "$lib rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_one.json')); d['lib']='$lib'; print(json.dumps(d))" >> gpurun_out/ab.jsonl
  python -c "import json; d=json.load(open('gpurun_out/ab_one.json')); r=d['roofline']; print('  ', d['ms_per_step'], r['kernel_ms'], r['frac'])"
done
