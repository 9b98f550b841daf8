#!/bin/bash
# fit parity tests + timing of the release and FIT_TIMING libraries (scripts/fit_prof.py)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/r03_fitab.txt
: > $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_api.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "invert or mll or update_k" >> $out 2>&1 || { echo "fit tests failed"; exit 1; }
for v in "" "_def_fit_waves=3" "_def_fit_timing"; do
  for c in C3 C5; do
    echo "== lib$v $c" >> $out
    BO_AMD_LIB=$PWD/bayesopt_smart_amd/libbo_amd$v.so timeout -k 10 200 python -u scripts/fit_prof.py $c 20 >> $out 2>&1 || exit 1
  done
done
echo done
