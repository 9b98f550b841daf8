#!/bin/bash
# HVI select A/B: the HVI GPU tests with the product library, then bench.py --acq hvi (C3) for
# each library in LIBS, interleaved twice; prints the hvi_select time of each run
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/hvi
timeout -k 10 300 python -u -m pytest tests/test_hvi.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/hvi/tests.log 2>&1 || { echo "hvi tests failed"; tail -20 gpurun_out/hvi/tests.log; exit 1; }
tail -1 gpurun_out/hvi/tests.log
for rnd in 1 2; do
  for lib in ${LIBS:-bayesopt_smart_amd/libbo_amd.so}; do
    n=$(basename $lib .so)
    BO_AMD_LIB=$R/$lib timeout -k 10 200 python bench.py --acq hvi --steps 20 --warmup 3 --no-cpu-baseline \
        > gpurun_out/hvi/${n}_$rnd.log 2>&1 || { echo "bench failed $n"; tail -5 gpurun_out/hvi/${n}_$rnd.log; exit 1; }
    python -c "import json; d=json.loads([l for l in open('gpurun_out/hvi/${n}_$rnd.log') if l.startswith('{')][-1]); h=d['hvi_select']; print('$n', $rnd, round(h['ms']*1e3,2), 'us', round(h['achieved_GBps'],1), 'GB/s', d['selected'])"
  done
done
