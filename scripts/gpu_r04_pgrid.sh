#!/bin/bash
# Persistent fit grid A/B (BO_FIT_PERSIST_GRID): MLL at C3 / C4, two rounds
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-r04q}
for round in 1 2; do
  for gr in 256 128 64 32; do
    for c in C3 C4; do
      BO_FIT_PERSIST_GRID=$gr timeout -k 10 300 python -u scripts/fit_prof.py $c 40 > gpurun_out/${TAG}_fp_${gr}_${c}_$round.txt 2>&1 \
        || { echo "fit prof $gr $c failed"; tail gpurun_out/${TAG}_fp_${gr}_${c}_$round.txt; exit 1; }
      echo "grid $gr $c r$round: $(grep -E '^mll|^inv' gpurun_out/${TAG}_fp_${gr}_${c}_$round.txt | tr '\n' ' ')"
    done
  done
done
