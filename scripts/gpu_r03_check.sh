#!/bin/bash
# Round-3 GPU check: the full -m gpu suite, smoke(), the default bench line (C3, strong scaling)
# and the fit timings.  Each step under its own time limit; stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-r03}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.jsonl 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; exit 1; }
timeout -k 10 300 python -u bench.py --fit --config C3 > gpurun_out/${TAG}_fit.jsonl 2>> gpurun_out/${TAG}_bench.err || { echo "fit failed"; exit 1; }
tail -2 gpurun_out/${TAG}_gpu_tests.log
echo done
