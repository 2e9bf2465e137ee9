#!/bin/bash
# Session 40: K3w row split: XCD alignment only when it adds no tile round (q|k|v at M = 16,000: 42 row ranges, 6 tiles each, instead of 40 with 7).

# then the text-tower GEMM shapes and the config-5 leg, base vs new, interleaved.
set -o pipefail
mkdir -p gpurun_out
P=${1:-r6s40}
L=multimodal-rag-for-image-text-search_amd/lib
for r in 0 1; do
  for lib in libmrag_base libmrag_rq; do
    MRAG_LIB=$L/$lib.so timeout -k 10 200 python -u scripts/gemm_roofline.py --only "clip_text:qkv,minilm:qkv" > gpurun_out/${P}_gemm_${lib}_${r}.jsonl 2> gpurun_out/${P}_gemm_${lib}_${r}.err || { echo "gemm $lib failed"; tail -20 gpurun_out/${P}_gemm_${lib}_${r}.err; exit 1; }
    python - $lib $r gpurun_out/${P}_gemm_${lib}_${r}.jsonl >> gpurun_out/${P}_gemm.jsonl <<'PY'
import json, sys
lib, r, path = sys.argv[1], sys.argv[2], sys.argv[3]
for l in open(path):
    if l.startswith("{"):
        d = json.loads(l); d["lib"] = lib; d["round"] = int(r); print(json.dumps(d))
PY
  done
done
grep -h '"us"\|us' gpurun_out/${P}_gemm.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['lib'], d['round'], d.get('tower'), d.get('gemm'), d.get("us"))"
for r in 0 1; do
  for lib in libmrag_base libmrag_rq; do
    MRAG_LIB=$L/$lib.so timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-clip --no-call-pattern --no-ingest --steps 20 --warmup 3 > gpurun_out/${P}_f_${lib}_${r}.log 2>&1 || { echo "fusion $lib failed"; tail -20 gpurun_out/${P}_f_${lib}_${r}.log; exit 1; }
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
