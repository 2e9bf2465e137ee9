#!/bin/bash
# Session 30: batches / steps in flight (at the box's hardware-queue setting).
# CLIP: 2..6 batches in flight, interleaved rounds; config 5: MRAG_FUSION_INFLIGHT 2 / 3 / 4 / 6
# through bench.py (other legs off), interleaved rounds.
set -o pipefail
mkdir -p gpurun_out
P=${1:-r6s30}
timeout -k 10 300 python -u scripts/clip_inflight_sweep.py --rounds 2 --steps 30 > gpurun_out/${P}_clip_inflight.jsonl 2> gpurun_out/${P}_clip_inflight.err || { echo "clip sweep failed"; tail -20 gpurun_out/${P}_clip_inflight.err; exit 1; }
cat gpurun_out/${P}_clip_inflight.jsonl
for r in 0 1; do
  for n in 2 3 4 6; do
    MRAG_FUSION_INFLIGHT=$n timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-clip --no-call-pattern --no-ingest --steps 20 --warmup 3 > gpurun_out/${P}_f${n}_${r}.log 2>&1 || { echo "fusion $n failed"; tail -20 gpurun_out/${P}_f${n}_${r}.log; exit 1; }
    python - "$n" "$r" gpurun_out/${P}_f${n}_${r}.log >> gpurun_out/${P}_fusion_inflight.jsonl <<'EOF'
import json, sys
n, r, path = sys.argv[1], sys.argv[2], sys.argv[3]
line = [l for l in open(path) if l.startswith('{"metric"')][-1]
d = json.loads(line)
f = d.get("fusion") or {}
print(json.dumps({"round": int(r), "fusion_inflight": int(n), "fusion_qps": f.get("value"),
                  "ms_per_step": f.get("ms_per_step"), "knn_qps": d["value"]}))
EOF
    tail -1 gpurun_out/${P}_fusion_inflight.jsonl
  done
done
