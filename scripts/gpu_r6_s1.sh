#!/bin/bash
# Round 6 session 1: the tests this round touched (RCCL world-1 gather, JPEG / PNG / ingest host
# half, compat), then the bench line with the new index_*_nodes legs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sharded_nccl_gpu.py tests/test_jpeg_gpu.py tests/test_png_gpu.py tests/test_compat_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r6s1_tests.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r6s1_tests.log; exit 3; }
tail -3 gpurun_out/r6s1_tests.log
timeout -k 10 900 python -u bench.py --no-cpu-baseline > gpurun_out/r6s1_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r6s1_bench.log; exit 5; }
grep '"metric"' gpurun_out/r6s1_bench.log | tail -1 > gpurun_out/r6s1_bench.json
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r6s1_bench.json"))
cp = d.get("call_pattern", {})
print("value", d["value"], "frac", d["roofline"]["frac"], "ms/step", d["ms_per_step"])
for k in ("index_image_nodes", "index_text_nodes", "ingest_embed_images_batch"):
    print(k, json.dumps(cp.get(k))[:900])
print("clip", d.get("clip", {}).get("value"), "fusion", d.get("fusion", {}).get("value"))
PY
