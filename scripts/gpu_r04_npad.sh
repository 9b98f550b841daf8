#!/bin/bash
# Last-chunk k-step skip: predict GPU tests, N-padding probe and C2/C3/C4 ablate A/B against the previous library
set -o pipefail
cd "$(dirname "$0")/.."
L=$PWD/bayesopt_smart_amd
TAG=${1:-r04np}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_predict.py tests/test_gpu_configs.py tests/test_gpu_api.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for lib in libbo_amd_prev.so libbo_amd.so; do
  BO_AMD_LIB=$L/$lib timeout -k 10 300 python -u scripts/npad_probe.py > gpurun_out/${TAG}_np_$lib.txt 2>&1 || { echo "probe $lib failed"; tail gpurun_out/${TAG}_np_$lib.txt; exit 1; }
  echo "== $lib"; grep "^N=" gpurun_out/${TAG}_np_$lib.txt
done
timeout -k 10 600 python -u scripts/ablate.py $L/libbo_amd_prev.so $L/libbo_amd.so cfg=C3 cfg=C2 cfg=C4 > gpurun_out/${TAG}_ablate.jsonl 2>&1 || { echo "ablate failed"; tail gpurun_out/${TAG}_ablate.jsonl; exit 1; }
grep median gpurun_out/${TAG}_ablate.jsonl
