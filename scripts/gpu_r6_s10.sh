#!/bin/bash
# Round 6 session 10: the coherent host flag instead of the per-search counter copy (kNN tests,
# same-box A/B against the previous library), and the batched index_image_nodes (its parity test
# and the bench's call-pattern legs).
P=r6s10
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py tests/test_compat_gpu.py tests/test_configs_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${P}_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${P}_tests.log; exit 3; }
tail -1 gpurun_out/${P}_tests.log
L=multimodal-rag-for-image-text-search_amd/lib
for r in 1 2 3; do
  for lib in libmrag_preflag libmrag; do
    MRAG_LIB=$R/$L/$lib.so timeout -k 10 300 python -u scripts/knn_scan_ab.py 30 > gpurun_out/${P}_ab_${lib}_$r.json 2>gpurun_out/${P}_ab_err.log || { echo "ab failed"; tail -5 gpurun_out/${P}_ab_err.log; exit 4; }
    echo "$lib $r $(tail -1 gpurun_out/${P}_ab_${lib}_$r.json)"
  done
done
timeout -k 10 900 python -u bench.py --no-cpu-baseline --no-clip --no-fusion > gpurun_out/${P}_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/${P}_bench.log; exit 5; }
grep '"metric"' gpurun_out/${P}_bench.log | tail -1 > gpurun_out/${P}_bench.json
python3 - gpurun_out/${P}_bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
cp = d.get("call_pattern", {})
print("knn", d["value"], "frac", d["roofline"]["frac"], "avg_launch_ms", d["roofline"]["avg_launch_ms"], "ms/step", d["ms_per_step"], "one", d["config"]["one_search_in_flight"])
for k in ("index_image_nodes", "index_text_nodes", "ingest_embed_images_batch", "retrieve", "device_q1"):
    print(k, json.dumps(cp.get(k))[:500])
PY
