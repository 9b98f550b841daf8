#!/bin/bash
# selection micro-benchmark (+ rocprofv3 kernel-trace of it): gpu_sel.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-sel}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python scripts/select_ubench.py > gpurun_out/${TAG}_ubench.jsonl 2> gpurun_out/${TAG}_ubench.err; rc=$?
echo "ubench rc=$rc"; cat gpurun_out/${TAG}_ubench.jsonl; tail -3 gpurun_out/${TAG}_ubench.err
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}" -o run -- \
    python "$R/scripts/select_ubench.py" --reps 20 > "$R/gpurun_out/prof_${TAG}.log" 2>&1; rc=$?
echo "prof rc=$rc"
exit $rc
