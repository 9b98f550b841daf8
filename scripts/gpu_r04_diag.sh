#!/bin/bash
# Round-4 diagnosis: persistent-fit phase stamps (C3, C5), the loop iteration's pieces.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-r04d}
for c in C3 C4 C5; do
  BO_AMD_LIB=$PWD/bayesopt_smart_amd/libbo_amd_def_fit_timing.so timeout -k 10 300 python -u scripts/fit_prof.py $c 20 \
    > gpurun_out/${TAG}_stamps_$c.txt 2>&1 || { echo "stamps $c failed"; tail gpurun_out/${TAG}_stamps_$c.txt; exit 1; }
  BO_FIT_PERSIST_MAX_NBT=999 BO_AMD_LIB=$PWD/bayesopt_smart_amd/libbo_amd_def_fit_timing.so timeout -k 10 300 \
    python -u scripts/fit_prof.py $c 20 > gpurun_out/${TAG}_stamps_p_$c.txt 2>&1 || { echo "stamps p $c failed"; exit 1; }
done
for c in C3 C5; do
  timeout -k 10 300 python -u scripts/lu_prof.py $c 680 10 > gpurun_out/${TAG}_lu_$c.txt 2>&1 || { echo "lu $c failed"; tail gpurun_out/${TAG}_lu_$c.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/${TAG}_lu_$c.txt
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_lu_prof -o lu -- python3 $GRAFT_REPO_ROOT/scripts/lu_prof.py C3 680 10) > gpurun_out/${TAG}_lu_prof.log 2>&1 || { echo "lu prof failed"; tail gpurun_out/${TAG}_lu_prof.log; exit 1; }
timeout -k 10 300 python -u scripts/iter_diag.py > gpurun_out/${TAG}_iter_diag.txt 2>&1 || { echo "iter diag failed"; tail gpurun_out/${TAG}_iter_diag.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_iter_diag.txt
for c in C3 C4 C5; do echo "== $c"; grep -v amdgpu.ids gpurun_out/${TAG}_stamps_$c.txt | head -4; echo "== $c (persistent at any N)"; grep -v amdgpu.ids gpurun_out/${TAG}_stamps_p_$c.txt | head -30; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp32.py -q -s --timeout 300 --timeout-method thread -k loop_iteration \
  > gpurun_out/${TAG}_fp32loop.log 2>&1; tail -5 gpurun_out/${TAG}_fp32loop.log; grep -E "float32 C5|max \|d acq" gpurun_out/${TAG}_fp32loop.log
