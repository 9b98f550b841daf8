#!/bin/bash
# Round-4 check: the GPU suite, then the device fit at C3/C4/C5 (bench.py --fit) and the default
# bench line.  Every GPU step under its own time limit; the first failure ends the script.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-r04}
# no -x: an assertion failure is reported and the measurements below still run; a GPU fault /
# abort / time limit (rc >= 124 or a crash) ends the script
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "gpu tests rc=$rc"; tail -40 gpurun_out/${TAG}_gpu_tests.log; exit 1; fi
grep -E "^FAILED|^ERROR" gpurun_out/${TAG}_gpu_tests.log || true
for c in C3 C4 C5; do
  timeout -k 10 300 python -u bench.py --fit --config $c >> gpurun_out/${TAG}_fit.jsonl 2> gpurun_out/${TAG}_fit_$c.err \
    || { echo "fit $c failed"; tail gpurun_out/${TAG}_fit_$c.err; exit 1; }
  # the same library on the launch-per-step schedule (same-box A/B)
  BO_FIT_PATH=launches timeout -k 10 300 python -u bench.py --fit --config $c >> gpurun_out/${TAG}_fit_launches.jsonl \
    2> gpurun_out/${TAG}_fit_l_$c.err || { echo "fit (launches) $c failed"; tail gpurun_out/${TAG}_fit_l_$c.err; exit 1; }
done
cat gpurun_out/${TAG}_fit_launches.jsonl
cat gpurun_out/${TAG}_fit.jsonl
if [ -z "${NO_EXTRA}" ]; then
  timeout -k 10 300 python -u bench.py --config C1 > gpurun_out/${TAG}_c1.jsonl 2> gpurun_out/${TAG}_c1.err \
    || { echo "C1 failed"; tail gpurun_out/${TAG}_c1.err; exit 1; }
  cat gpurun_out/${TAG}_c1.jsonl
  timeout -k 10 300 python -u bench.py --iteration --config C3 --steps 3 --warmup 1 > gpurun_out/${TAG}_iter_c3.jsonl \
    2> gpurun_out/${TAG}_iter_c3.err || { echo "iteration C3 failed"; tail gpurun_out/${TAG}_iter_c3.err; exit 1; }
  cat gpurun_out/${TAG}_iter_c3.jsonl
fi
if [ -z "${NO_BENCH}" ]; then
  timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.jsonl 2> gpurun_out/${TAG}_bench.err \
    || { echo "bench failed"; tail gpurun_out/${TAG}_bench.err; exit 1; }
  cat gpurun_out/${TAG}_bench.jsonl
fi
if [ -n "${ABLATE_LIBS}" ]; then
  timeout -k 10 600 python -u scripts/ablate.py bayesopt_smart_amd/libbo_amd.so ${ABLATE_LIBS} ${ABLATE_ARGS} \
    > gpurun_out/${TAG}_ablate.jsonl 2>&1 || { echo "ablate failed"; tail gpurun_out/${TAG}_ablate.jsonl; exit 1; }
  cat gpurun_out/${TAG}_ablate.jsonl
fi
