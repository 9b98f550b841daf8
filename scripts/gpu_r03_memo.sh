#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_api.py -m gpu -x -v -s --timeout 300 --timeout-method thread \
  -k "invert or mll or update_k or pivoting or powell or trajectory" > gpurun_out/r03_memo_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03_memo_tests.log; exit 1; }
for c in C3 C4 C5; do
  timeout -k 10 300 python -u bench.py --fit --config $c >> gpurun_out/r03c_fit.jsonl 2>> gpurun_out/r03c_fit.err || { echo "fit $c failed"; exit 1; }
done
echo done
