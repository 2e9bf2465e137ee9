#!/bin/bash
# Session 37: K7 with the query fragments landing under the first tile's MFMAs (first tile peeled,
# per-fragment waits, the seed used after the query loads are issued). kNN suites on the new
# library, then the kNN leg, base vs new, four interleaved rounds (order alternated).
set -o pipefail
mkdir -p gpurun_out
P=${1:-r6s37}
L=multimodal-rag-for-image-text-search_amd/lib
timeout -k 10 900 python -u -m pytest tests/test_knn_gpu.py tests/test_knn_generic_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${P}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${P}_tests.log; exit 1; }
tail -2 gpurun_out/${P}_tests.log
for r in 0 1 2 3; do
  if [ $((r % 2)) -eq 0 ]; then libs="libmrag_k7p libmrag_base"; else libs="libmrag_base libmrag_k7p"; fi
  for lib in $libs; do
    MRAG_LIB=$L/$lib.so timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-clip --no-fusion --no-call-pattern --no-ingest --steps 40 --warmup 5 > gpurun_out/${P}_${lib}_${r}.log 2>&1 || { echo "knn $lib failed"; tail -20 gpurun_out/${P}_${lib}_${r}.log; exit 1; }
    python - $lib $r gpurun_out/${P}_${lib}_${r}.log >> gpurun_out/${P}_knn.jsonl <<'PY'
import json, sys
lib, r, path = sys.argv[1], sys.argv[2], sys.argv[3]
d = json.loads([l for l in open(path) if l.startswith('{"metric"')][-1])
print(json.dumps({"lib": lib, "round": int(r), "value": d["value"], "ms_per_step": d["ms_per_step"],
                  "avg_launch_ms": d["roofline"]["avg_launch_ms"], "one": d["config"]["one_search_in_flight"],
                  "uncertified": d["config"]["uncertified_queries_last_step"]}))
PY
    tail -1 gpurun_out/${P}_knn.jsonl
  done
done
