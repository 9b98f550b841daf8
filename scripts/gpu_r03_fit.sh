#!/bin/bash
# Round-3 fit check: fit parity tests, the recorded select failure once under the bounds-checked
# library, and the fit timings (bench.py --fit) at C3/C4/C5.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_api.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "invert or mll or update_k" > gpurun_out/r03_fit_tests.log 2>&1 || { echo "fit tests failed"; exit 1; }
BO_AMD_LIB=$PWD/bayesopt_smart_amd/libbo_amd_def_debug_bounds.so timeout -k 10 300 python -u -m pytest \
  tests/test_gpu_api.py -m gpu -x -v --timeout 200 --timeout-method thread -k "select_exclusion_at_the_top" \
  > gpurun_out/r03_select_debug_bounds.log 2>&1 || { echo "debug select failed"; exit 1; }
for c in C3 C4 C5; do
  timeout -k 10 300 python -u bench.py --fit --config $c >> gpurun_out/r03_fit_bench.jsonl 2>> gpurun_out/r03_fit_bench.err || { echo "fit bench $c failed"; exit 1; }
done
echo done
