#!/bin/bash
# GPU predict parity tests, then kernel timings of the default library per mode.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_predict.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pred_tests.log 2>&1
rc=$?; tail -15 gpurun_out/pred_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ablate.py "$R/bayesopt_smart_amd/libbo_amd.so" ${ABL_LIBS} ${ABL_MODES:-mode=auto mode=dense} > gpurun_out/ablate.log 2>&1
rc=$?; grep median gpurun_out/ablate.log || tail -20 gpurun_out/ablate.log; exit $rc
