#!/bin/bash
# Round 5, session 4: hipGraph replay of small host-pointer token batches (retrieve's per-query
# encodes) and the pipelined ingest decode: encoder / compat / imgprep GPU tests, then the
# bench's retrieve and ingest legs (compare with r5s3).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py tests/test_compat_gpu.py tests/test_imgprep_gpu.py tests/test_embedder_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s4_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r5s4_tests.log; exit 3; }
tail -1 gpurun_out/r5s4_tests.log
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-clip --no-fusion > gpurun_out/r5s4_bench_legs.log 2>&1 || { echo "bench legs failed"; tail -30 gpurun_out/r5s4_bench_legs.log; exit 4; }
grep '"metric"' gpurun_out/r5s4_bench_legs.log | tail -1 > gpurun_out/r5s4_bench_legs.json
python3 -c "
import json; d=json.load(open('gpurun_out/r5s4_bench_legs.json'))
print(json.dumps(d.get('call_pattern',{}).get('retrieve'))); print(json.dumps(d.get('call_pattern',{}).get('ingest_embed_images_batch')))"
