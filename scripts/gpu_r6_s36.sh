#!/bin/bash
# Session 36: config-5 leg, base vs K3w-first-tile-overlap library, three more interleaved rounds
# (order alternated per round).
set -o pipefail
mkdir -p gpurun_out
P=${1:-r6s36}
L=multimodal-rag-for-image-text-search_amd/lib
for r in 0 1 2; do
  if [ $((r % 2)) -eq 0 ]; then libs="libmrag_wsw libmrag_base"; else libs="libmrag_base libmrag_wsw"; fi
  for lib in $libs; do
    MRAG_LIB=$L/$lib.so timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-clip --no-call-pattern --no-ingest --steps 30 --warmup 3 > gpurun_out/${P}_f_${lib}_${r}.log 2>&1 || { echo "fusion $lib failed"; tail -20 gpurun_out/${P}_f_${lib}_${r}.log; exit 1; }
    python - $lib $r gpurun_out/${P}_f_${lib}_${r}.log >> gpurun_out/${P}_fusion.jsonl <<'PY'
import json, sys
lib, r, path = sys.argv[1], sys.argv[2], sys.argv[3]
d = json.loads([l for l in open(path) if l.startswith('{"metric"')][-1])
f = d.get("fusion") or {}
print(json.dumps({"lib": lib, "round": int(r), "fusion_qps": f.get("value"), "one_step": (f.get("one_step_in_flight") or {}).get("queries_per_s"), "knn_qps": d["value"]}))
PY
    tail -1 gpurun_out/${P}_fusion.jsonl
  done
done
