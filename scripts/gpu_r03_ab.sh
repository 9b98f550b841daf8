#!/bin/bash
# Same-box A/B of library builds on the bench configs (fused-kernel time, scripts/ablate.py):
#   LIBS="a.so b.so" CFGS="C2 C3" bash scripts/gpu_r03_ab.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-ab}
LIBS=${LIBS:-$(ls bayesopt_smart_amd/libbo_amd*.so)}
CFGS=${CFGS:-C2 C3 C4}
args=""
for c in $CFGS; do args="$args cfg=$c"; done
timeout -k 10 600 python -u scripts/ablate.py $LIBS $args > gpurun_out/${TAG}.jsonl 2>&1 || { echo "ablate failed"; tail -20 gpurun_out/${TAG}.jsonl; exit 1; }
cat gpurun_out/${TAG}.jsonl
