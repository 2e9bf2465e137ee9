#!/bin/bash
# Round 6 validation of the current tree on one box (prefix $1): the full GPU suite, smoke, the
# driver's bench line.
P=${1:-r6v}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread > gpurun_out/${P}_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${P}_tests.log; exit 3; }
tail -1 gpurun_out/${P}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${P}_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/${P}_smoke.log; exit 4; }
tail -1 gpurun_out/${P}_smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/${P}_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/${P}_bench.log; exit 5; }
grep '"metric"' gpurun_out/${P}_bench.log | tail -1 > gpurun_out/${P}_bench.json
python3 - gpurun_out/${P}_bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
cp = d.get("call_pattern", {})
print("knn", d["value"], "frac", d["roofline"]["frac"], "avg_launch_ms", d["roofline"]["avg_launch_ms"], "ms/step", d["ms_per_step"], "one", d["config"]["one_search_in_flight"])
print("clip", d.get("clip", {}).get("value"), d.get("clip", {}).get("one_batch_in_flight"), "fusion", d.get("fusion", {}).get("value"))
for k in ("index_image_nodes", "index_text_nodes", "ingest_embed_images_batch", "retrieve"):
    print(k, json.dumps(cp.get(k))[:400])
print("cpu", json.dumps(d.get("cpu_baseline"))[:300])
PY
