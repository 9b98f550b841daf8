#!/bin/bash
# Fit tests, then MLL / inverse per path (persistent vs BO_FIT_PATH=launches) at C3/C4/C5 and the
# launch path's phase stamps at C5 (the FIT_TIMING build)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-r04i}
timeout -k 10 500 python -u -m pytest tests/test_gpu_fit.py tests/test_gpu_api.py tests/test_gpu_fit_launch_path.py -x -q --timeout 300 --timeout-method thread -k "mll or fit or powell or cobyla or persist or invert or launch" \
  > gpurun_out/${TAG}_fit_tests.log 2>&1 || { echo "fit tests failed"; tail -40 gpurun_out/${TAG}_fit_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_fit_tests.log
for c in ${CFGS:-C3 C4 C5}; do
  for path in persist launches; do
    BO_FIT_PATH=$path timeout -k 10 300 python -u scripts/fit_prof.py $c 30 > gpurun_out/${TAG}_fp_${path}_${c}.txt 2>&1 \
      || { echo "fit prof $path $c failed"; tail gpurun_out/${TAG}_fp_${path}_${c}.txt; exit 1; }
    echo "$c $path: $(grep -E '^mll|^inv' gpurun_out/${TAG}_fp_${path}_${c}.txt | tr '\n' ' ')"
  done
done
BO_AMD_LIB=$PWD/bayesopt_smart_amd/libbo_amd_def_fit_timing.so timeout -k 10 200 python -u scripts/fit_prof.py C5 20 > gpurun_out/${TAG}_stamps_C5.txt 2>&1 \
  || { echo "stamps failed"; exit 1; }
