#!/bin/bash
# Round-4 evidence, part A: the GPU suite, smoke, and every bench line from the shipped library.
# Each GPU step under its own limit; a crash / abort / time limit ends the script.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-r04_final}
O=gpurun_out/${TAG}
sha256sum bayesopt_smart_amd/libbo_amd.so > ${O}_lib_sha256.txt
if [ -z "${NO_TESTS}" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > ${O}_gpu_tests.log 2>&1
  rc=$?
  tail -2 ${O}_gpu_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "gpu tests rc=$rc"; tail -30 ${O}_gpu_tests.log; exit 1; fi
  grep -E "^FAILED|^ERROR" ${O}_gpu_tests.log || true
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > ${O}_smoke.log 2>&1 \
    || { echo "smoke failed"; tail ${O}_smoke.log; exit 1; }
  tail -1 ${O}_smoke.log
fi
run() {   # run NAME ARGS...: one bench line into ${O}_NAME.jsonl
  local name=$1; shift
  timeout -k 10 600 python -u bench.py "$@" > ${O}_${name}.jsonl 2> ${O}_${name}.err || { echo "bench $name failed"; tail ${O}_${name}.err; exit 1; }
  python - ${O}_${name}.jsonl "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
keys = ("value", "unit", "ms_per_step", "vs_baseline")
rf = d.get("roofline") or {}
print(sys.argv[2], {k: d.get(k) for k in keys}, "frac", rf.get("frac"), "traffic", rf.get("traffic"),
      "sel_cpu", d.get("selection_matches_cpu"), "cpu", (d.get("cpu_baseline") or {}).get("value"))
PY
}
[ -n "${NO_BENCH}" ] && exit 0
if [ "${SET:-1}" = "1" ]; then
  run c3_default
  run c2 --config C2
  run c4 --config C4
  run c5_fp32 --config C5
  run c5_f64 --config C5 --mode auto
else
  run c1 --config C1
  run iter_c3 --iteration --config C3 --steps 3 --warmup 1
  run iter_c5 --iteration --config C5 --steps 2 --warmup 1
  for c in C3 C4 C5; do run fit_$c --fit --config $c; done
  run c3_hvi --acq hvi
fi
