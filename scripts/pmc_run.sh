#!/bin/bash
# rocprofv3 PMC passes (one counter group per pass, kernel-trace only) over one command:
#   OUT=gpurun_out/pmc_X bash scripts/pmc_run.sh python3 bench.py --config C2 --steps 1 --warmup 1 --no-cpu-baseline
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:?set OUT}
mkdir -p "$R/$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$R/$OUT/p$i" -o run -- \
     "$@" > "$R/$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
