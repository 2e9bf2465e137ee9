#!/bin/bash
# Round 5, session 25: embed_images_batch with the GPU decode on its own thread and stream.
# The JPEG / PNG GPU tests (embed_images_batch equal with and without device decode), the group
# A/B and the bench's ingest leg.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_png_gpu.py tests/test_jpeg_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s25_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5s25_tests.log; exit 3; }
tail -1 gpurun_out/r5s25_tests.log
timeout -k 10 300 python3 -u scripts/ingest_group_ab.py 2048 > gpurun_out/r5s25_ingest_group_ab.jsonl 2>gpurun_out/r5s25.err || { echo "ab failed"; tail -5 gpurun_out/r5s25.err; exit 4; }
cat gpurun_out/r5s25_ingest_group_ab.jsonl
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-clip --no-fusion --no-retrieve-pattern > gpurun_out/r5s25_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r5s25_bench.log; exit 6; }
grep '"metric"' gpurun_out/r5s25_bench.log | tail -1 > gpurun_out/r5s25_bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/r5s25_bench.json'))
print(json.dumps(d.get('call_pattern',{}).get('ingest_embed_images_batch')))"
