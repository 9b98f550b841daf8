#!/bin/bash
# fit parity tests of each library in FITLIBS (suffixes of libbo_amd*.so, "" = the product), then
# the fit timing of each (scripts/fit_prof.py at C3 and C5)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-r03_fitab}
out=gpurun_out/${TAG}.txt
: > $out
for v in ${FITLIBS:-""}; do
  [ "$v" = "-" ] && v=""
  echo "== tests lib$v" >> $out
  BO_AMD_LIB=$PWD/bayesopt_smart_amd/libbo_amd$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_api.py -m gpu -x -q \
    --timeout 200 --timeout-method thread -k "invert or mll or update_k or powell or lu" >> $out 2>&1 || { echo "fit tests failed ($v)"; tail $out; exit 1; }
done
for rnd in 1 2; do
  for v in ${FITLIBS:-""}; do
    [ "$v" = "-" ] && v=""
    for c in C3 C5; do
      echo "== lib$v $c" >> $out
      BO_AMD_LIB=$PWD/bayesopt_smart_amd/libbo_amd$v.so timeout -k 10 200 python -u scripts/fit_prof.py $c 20 >> $out 2>&1 || exit 1
    done
  done
done
grep -E "^==|wall|passed|failed" $out
