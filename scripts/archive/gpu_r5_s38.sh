#!/bin/bash
# Round 5, session 38: the library host half at 8-32 threads alone and in embed_images_batch;
# the bench's ingest leg with its stage split.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 400 python3 -u scripts/ingest_native_threads.py 2048 > gpurun_out/r5s38_threads.jsonl 2> gpurun_out/r5s38.err || { echo "threads failed"; tail -20 gpurun_out/r5s38.err; exit 3; }
cat gpurun_out/r5s38_threads.jsonl
timeout -k 10 600 python3 -u bench.py --no-cpu-baseline --no-clip --no-fusion --no-retrieve-pattern --steps 5 > gpurun_out/r5s38_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r5s38_bench.log; exit 4; }
grep '"metric"' gpurun_out/r5s38_bench.log | tail -1 > gpurun_out/r5s38_bench.json
python3 -c "import json; d=json.load(open('gpurun_out/r5s38_bench.json')); print(json.dumps(d.get('call_pattern',{}).get('ingest_embed_images_batch'), indent=1))"
