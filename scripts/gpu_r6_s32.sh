#!/bin/bash
# Session 32: kNN searches in flight (--knn-streams 2 / 3 / 4) at the box's hardware-queue setting, interleaved
# rounds, kNN leg only.
set -o pipefail
mkdir -p gpurun_out
P=${1:-r6s32}
for r in 0 1; do
  for s in 2 3 4; do
    timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-clip --no-fusion --no-call-pattern --no-ingest --knn-streams $s --steps 40 --warmup 5 > gpurun_out/${P}_s${s}_${r}.log 2>&1 || { echo "knn $s failed"; tail -20 gpurun_out/${P}_s${s}_${r}.log; exit 1; }
    python - "$s" "$r" gpurun_out/${P}_s${s}_${r}.log >> gpurun_out/${P}_knn_streams.jsonl <<'PY'
import json, sys
s, r, path = sys.argv[1], sys.argv[2], sys.argv[3]
d = json.loads([l for l in open(path) if l.startswith('{"metric"')][-1])
print(json.dumps({"round": int(r), "knn_streams": int(s), "value": d["value"], "ms_per_step": d["ms_per_step"],
                  "avg_launch_ms": d["roofline"]["avg_launch_ms"],
                  "gap_ms": round(d["ms_per_step"] - d["roofline"]["avg_launch_ms"], 4)}))
PY
    tail -1 gpurun_out/${P}_knn_streams.jsonl
  done
done
