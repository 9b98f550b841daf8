#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in C3 C5; do
  timeout -k 10 200 python -u scripts/fit_prof.py $c 20 > gpurun_out/r03_fitprof_$c.txt 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fit_$c -o fit -- python3 scripts/fit_prof.py $c 20 > gpurun_out/r03_fitprof_${c}_rocprof.log 2>&1 || exit 1
done
echo done
