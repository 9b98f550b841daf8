#!/bin/bash
# The fused predict at N = 512, 518 and 530 (PART: padded last chunk) and 544 (full padding), for each
# library build in LIBS (default: every libbo_amd*.so), after a sha256 of each build's
# outputs at N = 518, 524 and 530 (bit-for-bit comparison).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
LIBS=${LIBS:-$(cd bayesopt_smart_amd && ls libbo_amd*.so)}
for lib in $LIBS; do
  echo "lib=$lib"
  for n in 518 524 530; do
    BO_AMD_LIB=$R/bayesopt_smart_amd/$lib timeout -k 10 180 python scripts/part_compare.py $n  || exit $?
  done
  for n in 512 518 530 544; do
    echo "lib=$lib"
    BO_AMD_LIB=$R/bayesopt_smart_amd/$lib timeout -k 10 180 python scripts/outputs_probe.py $n || exit $?
  done
done
