#!/bin/bash
# C5 bench lines (f64 and the stated fp32) with the whole 4M-candidate shard scored by the CPU
# reference outside the timed region, so that selection_matches_cpu is decided (not null)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/c5full
: > gpurun_out/c5full/bench.jsonl
for m in auto fp32; do
  timeout -k 10 500 python bench.py --config C5 --mode $m --steps 3 --warmup 2 --cpu-full \
      > gpurun_out/c5full/$m.json 2> gpurun_out/c5full/$m.err || { echo "fail $m"; tail -5 gpurun_out/c5full/$m.err; exit 1; }
  grep '^{' gpurun_out/c5full/$m.json | tail -1 >> gpurun_out/c5full/bench.jsonl
  python -c "import json; d=json.loads(open('gpurun_out/c5full/bench.jsonl').readlines()[-1]); print('$m', d['value'], d['dtype'], 'acq_err', d.get('acq_max_err_vs_cpu'), 'selection_matches_cpu', d.get('selection_matches_cpu'), d['selected'], d.get('cpu_selected'))"
done
