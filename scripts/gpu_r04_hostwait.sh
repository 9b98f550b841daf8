#!/bin/bash
# MLL host wait A/B: pinned completion-word polling (default) vs stream synchronisation
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-r04n}
timeout -k 10 500 python -u -m pytest tests/test_gpu_fit.py tests/test_gpu_api.py tests/test_gpu_fit_launch_path.py -x -q --timeout 300 --timeout-method thread -k "mll or fit or powell or cobyla or persist or invert or launch" \
  > gpurun_out/${TAG}_fit_tests.log 2>&1 || { echo "fit tests failed"; tail -40 gpurun_out/${TAG}_fit_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_fit_tests.log
for round in 1 2; do
  for w in sync poll; do
    for c in C3 C4; do
      BO_FIT_HOSTWAIT=$w timeout -k 10 300 python -u scripts/fit_prof.py $c 40 > gpurun_out/${TAG}_fp_${w}_${c}_$round.txt 2>&1 \
        || { echo "fit prof $w $c failed"; tail gpurun_out/${TAG}_fp_${w}_${c}_$round.txt; exit 1; }
      echo "$w $c r$round: $(grep -E '^mll' gpurun_out/${TAG}_fp_${w}_${c}_$round.txt)"
    done
    BO_FIT_HOSTWAIT=$w timeout -k 10 300 python -u bench.py --fit --config C3 > gpurun_out/${TAG}_fit_${w}_$round.jsonl 2>/dev/null || { echo "bench fit failed"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'powell ms', round(d['value'],3), 'per eval', round(d['powell_ms_per_eval'],4), 'mll', round(d['compute_mll_ms'],4), d['fit_paths_during_powell'])" gpurun_out/${TAG}_fit_${w}_$round.jsonl $w
  done
done
