#!/bin/bash
# Full GPU suite, then a same-box A/B of the product library against LIBS on CFGS.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-full}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_gpu_tests.log
if [ -n "${CFGS}" ]; then
  args=""
  for c in $CFGS; do args="$args cfg=$c"; done
  timeout -k 10 900 python -u scripts/ablate.py bayesopt_smart_amd/libbo_amd.so ${LIBS} $args ${ABL_ARGS} > gpurun_out/${TAG}_ab.jsonl 2>&1 || { echo "ablate failed"; tail gpurun_out/${TAG}_ab.jsonl; exit 1; }
  cat gpurun_out/${TAG}_ab.jsonl
fi
