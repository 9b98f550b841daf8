#!/bin/bash
# rocprofv3 kernel stats of the selection micro-benchmark: gpu_prof_sel.sh TAG CASES [LIB]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; CASES=$2; LIB=${3:-bayesopt_smart_amd/libbo_amd.so}
export TMPDIR=/tmp BO_AMD_LIB=$R/$LIB
cd /tmp
for c in ${CASES//,/ }; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/profsel_${TAG}_$c" -o run -- \
      python3 "$R/scripts/select_ubench.py" --cases $c --reps 20 > "$R/gpurun_out/profsel_${TAG}_$c.log" 2>&1 || exit 1
  f=$(find "$R/gpurun_out/profsel_${TAG}_$c" -name "*kernel_stats.csv" | head -1)
  echo "== $c"; cut -d, -f1-4 "$f" | head -6
done
