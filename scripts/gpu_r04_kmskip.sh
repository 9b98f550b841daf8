#!/bin/bash
# Fit without per-evaluation kernel-matrix writes: fit tests, then the native Powell fit at C3 / C5
# (scripts/trig_probe.py, numpy_trig lines) for the previous library and this one, interleaved
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-r04u}
timeout -k 10 500 python -u -m pytest tests/test_gpu_fit.py tests/test_gpu_api.py tests/test_gpu_fit_launch_path.py tests/test_gpu_fp32.py -x -q --timeout 300 --timeout-method thread -k "mll or fit or powell or cobyla or persist or invert or launch or memo or float32" \
  > gpurun_out/${TAG}_fit_tests.log 2>&1 || { echo "fit tests failed"; tail -40 gpurun_out/${TAG}_fit_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_fit_tests.log
for round in 1 2; do
  for lib in libbo_amd_prev.so libbo_amd.so; do
    for c in C3 C5; do
      BO_AMD_LIB=$PWD/bayesopt_smart_amd/$lib timeout -k 10 300 python -u scripts/trig_probe.py $c > gpurun_out/${TAG}_fit_${lib}_${c}_$round.txt 2>&1 || { echo "probe failed"; tail gpurun_out/${TAG}_fit_${lib}_${c}_$round.txt; exit 1; }
      echo "$lib $c r$round: $(grep 'numpy_trig=True' gpurun_out/${TAG}_fit_${lib}_${c}_$round.txt | tail -2 | tr '\n' ' ')"
    done
  done
done
