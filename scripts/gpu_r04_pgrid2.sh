#!/bin/bash
# Persistent grid heuristic vs the fixed 256: fit tests, MLL at C3 / C4, the C3 Powell fit
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-r04r}
timeout -k 10 500 python -u -m pytest tests/test_gpu_fit.py tests/test_gpu_api.py tests/test_gpu_fit_launch_path.py -x -q --timeout 300 --timeout-method thread -k "mll or fit or powell or cobyla or persist or invert or launch" \
  > gpurun_out/${TAG}_fit_tests.log 2>&1 || { echo "fit tests failed"; tail -40 gpurun_out/${TAG}_fit_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_fit_tests.log
for round in 1 2; do
  for gr in 256 0; do
    for c in C3 C4; do
      BO_FIT_PERSIST_GRID=$gr timeout -k 10 300 python -u scripts/fit_prof.py $c 40 > gpurun_out/${TAG}_fp_${gr}_${c}_$round.txt 2>&1 \
        || { echo "fit prof $gr $c failed"; exit 1; }
      echo "grid $gr $c r$round: $(grep -E '^mll' gpurun_out/${TAG}_fp_${gr}_${c}_$round.txt)"
    done
    BO_FIT_PERSIST_GRID=$gr timeout -k 10 300 python -u bench.py --fit --config C3 > gpurun_out/${TAG}_fit_${gr}_$round.jsonl 2>/dev/null || { echo "bench fit failed"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('grid', sys.argv[2], 'powell ms', round(d['value'],3), 'mll', round(d['compute_mll_ms'],4))" gpurun_out/${TAG}_fit_${gr}_$round.jsonl $gr
  done
done
