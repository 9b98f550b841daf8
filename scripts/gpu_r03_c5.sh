#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_c5_shards.py -m gpu -x -v -s --timeout 600 --timeout-method thread \
  > gpurun_out/r03_c5_shards.log 2>&1 || { echo "c5 shard tests failed"; tail -30 gpurun_out/r03_c5_shards.log; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/r03b_bench.jsonl 2> gpurun_out/r03b_bench.err || { echo "bench failed"; exit 1; }
echo done
