#!/bin/bash
# LU fallback tests + the C5 shard parity + bench line + fit timings (C3, C5) + demo-style
# fallback frequency.  Stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_api.py -m gpu -x -v -s --timeout 300 --timeout-method thread \
  -k "invert or mll or update_k or pivoting" > gpurun_out/r03_lu_tests.log 2>&1 || { echo "lu tests failed"; tail -40 gpurun_out/r03_lu_tests.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_c5_shards.py -m gpu -x -v -s --timeout 600 --timeout-method thread \
  > gpurun_out/r03_c5_shards.log 2>&1 || { echo "c5 shard tests failed"; tail -40 gpurun_out/r03_c5_shards.log; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/r03b_bench.jsonl 2> gpurun_out/r03b_bench.err || { echo "bench failed"; exit 1; }
for c in C3 C5; do
  timeout -k 10 300 python -u bench.py --fit --config $c >> gpurun_out/r03b_fit.jsonl 2>> gpurun_out/r03b_bench.err || { echo "fit $c failed"; exit 1; }
done
timeout -k 10 600 python -u bench.py --fit-demo 512 > gpurun_out/r03b_fit_demo.json 2>> gpurun_out/r03b_bench.err || { echo "fit demo failed"; exit 1; }
echo done
