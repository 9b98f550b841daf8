#!/bin/bash
# Launch-path fit A/B over several libraries (interleaved, 2 rounds): MLL and inverse at N = 2048
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-r04h}
LIBS=${LIBS:-"libbo_amd_prev.so libbo_amd.so"}
CFG=${CFG:-C5}
for round in 1 2; do
  for lib in $LIBS; do
    BO_AMD_LIB=$PWD/bayesopt_smart_amd/$lib timeout -k 10 300 python -u scripts/fit_prof.py $CFG 30 > gpurun_out/${TAG}_fp_${lib}_${CFG}_$round.txt 2>&1 \
      || { echo "fit prof $lib failed"; tail gpurun_out/${TAG}_fp_${lib}_${CFG}_$round.txt; exit 1; }
    echo "$lib r$round: $(grep -E '^mll|^inv' gpurun_out/${TAG}_fp_${lib}_${CFG}_$round.txt | tr '\n' ' ')"
  done
done
