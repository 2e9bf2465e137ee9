#!/bin/bash
# Round 5, session 3: the new bench legs (per-query retrieve_text / retrieve_images through the
# drop-in, embed_images_batch from image files) on one GPU, and bench.py's N = 2 path rehearsed on
# one GPU over gloo: the line must say backend gloo, world 2 (numbers are two ranks sharing a GPU).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-clip --no-fusion > gpurun_out/r5s3_bench_legs.log 2>&1 || { echo "bench legs failed"; tail -30 gpurun_out/r5s3_bench_legs.log; exit 3; }
grep '"metric"' gpurun_out/r5s3_bench_legs.log | tail -1 > gpurun_out/r5s3_bench_legs.json
python3 -c "
import json; d=json.load(open('gpurun_out/r5s3_bench_legs.json'))
print(json.dumps(d.get('call_pattern',{}).get('retrieve'))); print(json.dumps(d.get('call_pattern',{}).get('ingest_embed_images_batch')))"
export MRAG_DIST_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-clip > gpurun_out/r5s3_bench_n2_gloo.log 2>&1 || { echo "bench n2 failed"; tail -20 gpurun_out/r5s3_bench_n2_gloo.log; exit 4; }
grep '"metric"' gpurun_out/r5s3_bench_n2_gloo.log | tail -1 > gpurun_out/r5s3_bench_n2_gloo.json
python3 -c "
import json; d=json.load(open('gpurun_out/r5s3_bench_n2_gloo.json'))
print(d['value'], d['config']['parallelism']); print(json.dumps(d.get('comm')))"
