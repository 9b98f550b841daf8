#!/bin/bash
# Functional rehearsal of bench.py's multi-rank step on ONE device (gloo exchange, P ranks
# sharing cuda:0; not a measurement): each config at 1 rank, then 2 and 4 ranks through
# torch.distributed.run; the selected batch must be the same at every P.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/dist
out=gpurun_out/dist/rehearsal.jsonl
: > $out
port=29511
for c in ${CFGS:-C3 C4}; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/dist/${c}_p1.log 2>&1 || { echo "fail $c p1"; tail -5 gpurun_out/dist/${c}_p1.log; exit 1; }
  grep '^{' gpurun_out/dist/${c}_p1.log | tail -1 >> $out
  for p in 2 4; do
    port=$((port + 1))
    BO_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $p \
        --master-addr 127.0.0.1 --master-port $port bench.py --gpus $p --config $c --steps 3 --warmup 1 \
        > gpurun_out/dist/${c}_p$p.log 2>&1 || { echo "fail $c p$p"; tail -5 gpurun_out/dist/${c}_p$p.log; exit 1; }
    grep '^{' gpurun_out/dist/${c}_p$p.log | tail -1 >> $out
  done
done
python - "$out" <<'EOF'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
ok = True
for r in rows:
    c = r["config"]
    base = next(x for x in rows if x["config"]["workload"] == c["workload"] and x["n_gpus"] == 1)
    same = r["selected"] == base["selected"]
    ok &= same
    ro = r.get("roofline", {})
    ss = r.get("select_standalone") or {}
    local_ok = ss.get("matches_fused_selection")
    ok &= local_ok is not False
    print(c["workload"][:3], "P =", r["n_gpus"], "per rank", c["n_cand_per_gpu"], "offset(rank 0)", c["candidate_offset"],
          "selected", r["selected"], "same as P=1:", same, "| traffic", ro.get("traffic"), "ratio",
          ro.get("traffic_ratio"), "| select_standalone vs the rank-local fused selection:", local_ok,
          "| collectives", r.get("collectives"))
print("all equal:", ok)
sys.exit(0 if ok else 1)
EOF
