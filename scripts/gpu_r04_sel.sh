#!/bin/bash
# Standalone selection: GPU tests, A/B ubench against the round-start library (interleaved),
# phase stamps (DEF_SEL_TIMING)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-r04s}
timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py -x -q --timeout 200 --timeout-method thread -k "select or hvi or exclusion" \
  > gpurun_out/${TAG}_sel_tests.log 2>&1 || { echo "select tests failed"; tail -30 gpurun_out/${TAG}_sel_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_sel_tests.log
for round in 1 2; do
  for lib in libbo_amd_r04base.so libbo_amd.so; do
    BO_AMD_LIB=$PWD/bayesopt_smart_amd/$lib timeout -k 10 300 python -u scripts/select_ubench.py --cases C3,C3noex,C2,C5 \
      > gpurun_out/${TAG}_ub_${lib}_$round.jsonl 2>/dev/null || { echo "ubench $lib failed"; exit 1; }
    echo "$lib round $round: $(python -c "import json,sys; print(' '.join(f\"{d['case']}={d['us_per_call']}\" for d in map(json.loads, open(sys.argv[1]))))" gpurun_out/${TAG}_ub_${lib}_$round.jsonl)"
  done
done
BO_AMD_LIB=$PWD/bayesopt_smart_amd/libbo_amd_def_sel_timing.so timeout -k 10 120 python -u scripts/select_ubench.py --cases C3 --reps 1 \
  > gpurun_out/${TAG}_stamps.txt 2>&1 || { echo "stamps failed"; tail gpurun_out/${TAG}_stamps.txt; exit 1; }
grep "sel block" gpurun_out/${TAG}_stamps.txt | tail -4
