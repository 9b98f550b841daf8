#!/bin/bash
# Round evidence in one GPU session: parity tests + smoke, PMC summaries (C2, C3, C4), the
# per-config bench lines, rocprofv3 kernel stats of the C3 headline.  Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r02_final}
bash scripts/gpu_check.sh tests || exit $?
bash scripts/gpu_check.sh smoke || exit $?
for c in C2 C3 C4; do
  CONFIG=$c bash scripts/pmc_cfg.sh > gpurun_out/pmc_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
  k="cm_predict_kernel<2, true, true, false, 4>"; alg=$((8*5*262144))
  [ $c = C3 ] && { k="cm_predict_kernel<2, true, true, false, 16>"; alg=$((8*5*1048576)); }
  [ $c = C4 ] && { k="cm_predict_kernel<6, false, true, false, 16>"; alg=$((8*(7+6)*2097152)); }
  python scripts/pmc_summary.py gpurun_out/pmc_$c gpurun_out/${TAG}_${c,,}_pmc.json $c $alg "$k" > /dev/null || exit 1
  cp gpurun_out/${TAG}_${c,,}_pmc.json profiles/ 
done
bash scripts/gpu_configs_bench.sh > gpurun_out/configs.log 2>&1; rc=$?; cat gpurun_out/configs.log; [ $rc -eq 0 ] || exit $rc
bash scripts/prof_cfg.sh ${TAG} C3
