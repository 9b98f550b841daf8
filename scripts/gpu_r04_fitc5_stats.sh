#!/bin/bash
# rocprofv3 kernel stats of the C5 fit (launch-per-step path: fit_step_kernel<SPLIT, UPD>)
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
TAG=${1:-r04b_final}
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_st_fit5 -o run -- python3 $R/bench.py --fit --config C5) \
  > gpurun_out/${TAG}_st_fit5.log 2>&1 || { echo "stats failed"; tail gpurun_out/${TAG}_st_fit5.log; exit 1; }
f=$(find gpurun_out/${TAG}_st_fit5 -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${TAG}_fit5_kernel_stats.csv
cut -d, -f1-4 gpurun_out/${TAG}_fit5_kernel_stats.csv | head -12
