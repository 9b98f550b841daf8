#!/bin/bash
# Selection kernels: the select / HVI / predict GPU tests, then the standalone selection
# micro-benchmark for the product library and each library named in LIBS.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-sel}
timeout -k 10 600 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_configs.py tests/test_hvi.py tests/test_gpu_predict.py \
  -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
: > gpurun_out/${TAG}_ubench.jsonl
for lib in bayesopt_smart_amd/libbo_amd.so ${LIBS}; do
  echo "== $lib" >> gpurun_out/${TAG}_ubench.jsonl
  BO_AMD_LIB=$(pwd)/$lib timeout -k 10 180 python -u scripts/select_ubench.py >> gpurun_out/${TAG}_ubench.jsonl 2>&1 || { echo "ubench failed"; exit 1; }
done
cat gpurun_out/${TAG}_ubench.jsonl
