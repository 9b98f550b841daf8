#!/bin/bash
# Fit A/B: the fit GPU tests, MLL / inverse timing per library (interleaved), phase stamps (C3)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-r04f}
B=${BASE_LIB:-libbo_amd_prev.so}
timeout -k 10 500 python -u -m pytest tests/test_gpu_fit.py tests/test_gpu_api.py -x -q --timeout 300 --timeout-method thread -k "mll or fit or powell or cobyla or persist or invert" \
  > gpurun_out/${TAG}_fit_tests.log 2>&1 || { echo "fit tests failed"; tail -40 gpurun_out/${TAG}_fit_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_fit_tests.log
for round in 1 2; do
  for lib in $B libbo_amd.so; do
    for c in C3 C5; do
      BO_AMD_LIB=$PWD/bayesopt_smart_amd/$lib timeout -k 10 300 python -u scripts/fit_prof.py $c 30 > gpurun_out/${TAG}_fp_${lib}_${c}_$round.txt 2>&1 \
        || { echo "fit prof $lib $c failed"; tail gpurun_out/${TAG}_fp_${lib}_${c}_$round.txt; exit 1; }
      echo "$lib r$round: $(grep -E '^mll|^inv' gpurun_out/${TAG}_fp_${lib}_${c}_$round.txt | tr '\n' ' ')"
    done
  done
done
BO_AMD_LIB=$PWD/bayesopt_smart_amd/libbo_amd_def_fit_timing.so timeout -k 10 200 python -u scripts/fit_prof.py C3 20 > gpurun_out/${TAG}_stamps_C3.txt 2>&1 \
  || { echo "stamps failed"; exit 1; }
grep -E "^k (0|1|2|8|15) " gpurun_out/${TAG}_stamps_C3.txt
if [ -n "${POWELL}" ]; then
  for lib in $B libbo_amd.so; do
    BO_AMD_LIB=$PWD/bayesopt_smart_amd/$lib timeout -k 10 300 python -u bench.py --fit --config C3 > gpurun_out/${TAG}_fit_${lib}.jsonl 2>/dev/null || { echo "bench fit failed"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k: v for k, v in d.items() if 'ms' in k or 'fit' in k})" gpurun_out/${TAG}_fit_${lib}.jsonl $lib
  done
fi
if [ -n "${PROF}" ]; then
  for lib in $B libbo_amd.so; do
    (cd /tmp && export TMPDIR=/tmp && BO_AMD_LIB=$GRAFT_REPO_ROOT/bayesopt_smart_amd/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_$lib -o fit -- python3 $GRAFT_REPO_ROOT/scripts/fit_prof.py C3 30) > gpurun_out/${TAG}_prof_$lib.log 2>&1 || { echo "prof $lib failed"; tail gpurun_out/${TAG}_prof_$lib.log; exit 1; }
    f=$(find gpurun_out/${TAG}_prof_$lib -name "*kernel_stats.csv" | head -1)
    echo "== $lib"; python - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print("  ", r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
  done
fi
