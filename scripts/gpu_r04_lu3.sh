#!/bin/bash
# LU fallback: tests, timing (default library), per-column panel stamps (diagnostic library)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-r04j}
timeout -k 10 400 python -u -m pytest tests/test_gpu_api.py -x -v -s --timeout 300 --timeout-method thread -k "lu or invert" \
  > gpurun_out/${TAG}_lu_tests.log 2>&1 || { echo "LU tests failed"; tail -40 gpurun_out/${TAG}_lu_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/${TAG}_lu_tests.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_fit.py tests/test_gpu_api.py -x -q --timeout 300 --timeout-method thread -k "mll or fit or powell or cobyla or persist" \
  > gpurun_out/${TAG}_fit_tests.log 2>&1 || { echo "fit tests failed"; tail -40 gpurun_out/${TAG}_fit_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_fit_tests.log
for c in C3 C5; do
  timeout -k 10 300 python -u scripts/fit_prof.py $c 30 > gpurun_out/${TAG}_fitprof_$c.txt 2>&1 || { echo "fit prof $c failed"; exit 1; }
  grep -E "^mll|^inv" gpurun_out/${TAG}_fitprof_$c.txt
done
for c in C3 C4 C5; do
  timeout -k 10 300 python -u scripts/lu_prof.py $c 680 10 > gpurun_out/${TAG}_lu_$c.txt 2>&1 || { echo "lu $c failed"; tail gpurun_out/${TAG}_lu_$c.txt; exit 1; }
  grep invert_k gpurun_out/${TAG}_lu_$c.txt
done
BO_AMD_LIB=$PWD/bayesopt_smart_amd/libbo_amd_def_fit_timing.so timeout -k 10 300 python -u scripts/lu_prof.py C3 680 3 \
  > gpurun_out/${TAG}_lu_stamps_C3.txt 2>&1 || { echo "lu stamps failed"; tail gpurun_out/${TAG}_lu_stamps_C3.txt; exit 1; }
grep -E "^step [0-3] |^solve [0-3] " gpurun_out/${TAG}_lu_stamps_C3.txt
grep -A17 "panel step 1" gpurun_out/${TAG}_lu_stamps_C3.txt
BO_AMD_LIB=$PWD/bayesopt_smart_amd/libbo_amd_def_fit_timing.so timeout -k 10 300 python -u scripts/lu_prof.py C5 680 2 \
  > gpurun_out/${TAG}_lu_stamps_C5.txt 2>&1 || { echo "lu stamps C5 failed"; tail gpurun_out/${TAG}_lu_stamps_C5.txt; exit 1; }
grep -E "^step [0-3] |^solve [0-3] " gpurun_out/${TAG}_lu_stamps_C5.txt
grep -A6 "panel step 1" gpurun_out/${TAG}_lu_stamps_C5.txt
